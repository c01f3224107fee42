#!/usr/bin/env python3
"""Two-process HIP IPC probe: the mechanism RCCL's P2P/IPC transport maps a peer GPU's buffers with
(hipIpcGetMemHandle in the owner, hipIpcOpenMemHandle in the peer).  On an 8-GPU node the flat
schedule's ncclSend/ncclRecv between ranks go over xGMI through it; on this host driver it works only
with dmabuf IPC (HSA_ENABLE_IPC_MODE_LEGACY=0, which bench.py and chiara_amd set before HIP loads).

  ipc_probe.py owner NBYTES   allocate, fill word i with i ^ 0x5A5A0000, print the 64-byte handle as
                              hex, wait for one line on stdin, check the peer's writes, print OK
  ipc_probe.py peer HEX NBYTES  open the handle, check the owner's words, overwrite word i with ~i,
                              print OK

Plain ctypes over torch's libamdhip64 (the same HIP runtime the product links); no torch.cuda call, so
nothing but these HIP calls touches the GPU.  Used by tests/test_gpu_ipc.py."""
import ctypes
import os
import sys

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


class IpcHandle(ctypes.Structure):
    """hipIpcMemHandle_t: 64 opaque bytes, passed BY VALUE to hipIpcOpenMemHandle (a ctypes array argtype
    would be passed as a pointer)."""
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hip():
    import torch  # only to locate its libamdhip64 (one HIP runtime per process)

    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    lib.hipFree.argtypes = [vp]
    lib.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
    lib.hipIpcGetMemHandle.argtypes = [ctypes.c_char_p, vp]
    lib.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), IpcHandle, ctypes.c_uint]
    lib.hipIpcCloseMemHandle.argtypes = [vp]
    lib.hipSetDevice.argtypes = [ctypes.c_int]
    return lib


H2D, D2H = 1, 2


def ck(rc, what):
    if rc != 0:
        print(f"FAIL {what} rc={rc}", flush=True)
        sys.exit(3)


def words(n, kind):
    """The probe's word patterns as a contiguous uint32 array: "owner" i ^ 0x5A5A0000, "peer" ~i, "zero"."""
    import numpy as np

    i = np.arange(n, dtype=np.uint32)
    return {"owner": i ^ np.uint32(0x5A5A0000), "peer": ~i, "zero": np.zeros(n, dtype=np.uint32)}[kind]


def main():
    mode = sys.argv[1]
    lib = hip()
    ck(lib.hipSetDevice(0), "hipSetDevice")
    if mode == "owner":
        nbytes = int(sys.argv[2])
        n = nbytes // 4
        p = ctypes.c_void_p()
        ck(lib.hipMalloc(ctypes.byref(p), nbytes), "hipMalloc")
        src = words(n, "owner")
        ck(lib.hipMemcpy(p, src.ctypes.data, nbytes, H2D), "hipMemcpy H2D")
        h = ctypes.create_string_buffer(64)
        ck(lib.hipIpcGetMemHandle(h, p), "hipIpcGetMemHandle")
        print(h.raw.hex(), flush=True)
        sys.stdin.readline()  # the peer has written
        back = words(n, "zero")
        ck(lib.hipMemcpy(back.ctypes.data, p, nbytes, D2H), "hipMemcpy D2H")
        want = words(n, "peer")
        ok = bool((back == want).all())
        print("OK" if ok else f"FAIL owner sees {back[:4].tolist()} want {want[:4].tolist()}", flush=True)
        ck(lib.hipFree(p), "hipFree")
    else:
        hx, nbytes = sys.argv[2], int(sys.argv[3])
        n = nbytes // 4
        h = IpcHandle.from_buffer_copy(bytes.fromhex(hx))
        p = ctypes.c_void_p()
        ck(lib.hipIpcOpenMemHandle(ctypes.byref(p), h, 1), "hipIpcOpenMemHandle")  # hipIpcMemLazyEnablePeerAccess
        got = words(n, "zero")
        ck(lib.hipMemcpy(got.ctypes.data, p, nbytes, D2H), "hipMemcpy D2H (peer)")
        if not (got == words(n, "owner")).all():
            print(f"FAIL peer sees {got[:4].tolist()}", flush=True)
            sys.exit(4)
        new = words(n, "peer")
        ck(lib.hipMemcpy(p, new.ctypes.data, nbytes, H2D), "hipMemcpy H2D (peer)")
        ck(lib.hipIpcCloseMemHandle(p), "hipIpcCloseMemHandle")
        print("OK", flush=True)


if __name__ == "__main__":
    main()
