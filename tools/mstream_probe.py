#!/usr/bin/env python3
"""Why m = 3 / m = 7 buckets drop at >= 512 MiB: the product's fused bucket
reduction (chr_reduce_multi, in place, fp32 SUM) at m in {1, 3, 7} incoming buckets and bucket
sizes 256 MiB .. 1 GiB, with the m + 1 operands laid out four ways:
  sep      one torch allocation per operand (the earlier sweep's layout)
  slab     one allocation, operands back to back (operand j at j * bucket)
  slab+d   one allocation, operand j at j * (bucket + d): d = 4 KiB, 64 KiB, 2 MiB + 4 KiB, and
           64 / 96 / 192 / 320 MiB (moving the operands' high address bits apart)
  contig   one hipExtMallocWithFlags(hipDeviceMallocContiguous) per operand (physically contiguous:
           can the page tables map it with larger fragments?)
  sep/sN   as sep, but each call issued as N back-to-back launches over consecutive 1/N pieces
           (bounds how far the in-flight workgroups of one launch can drift apart)
HBM-cold: at least 2 GiB of distinct data per rotation (buffer sets cycled).  Prints one JSON line
per (m, bucket, layout): us per call and algorithmic GB/s ((m + 2) * bucket bytes).
Usage: mstream_probe.py [--ms 1,3,7] [--mib 256,512,1024] [--layouts sep,slab,...] [--reps N] [--sets 1,2,4]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import ctypes  # noqa: E402

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

DELTAS = {"slab": 0, "slab+4k": 4 << 10, "slab+64k": 64 << 10, "slab+2m4k": (2 << 20) + (4 << 10),
          "slab+64m": 64 << 20, "slab+192m": 192 << 20, "slab+320m": 320 << 20, "slab+96m4k": (96 << 20) + (4 << 10)}


def _hip():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    lib.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    lib.hipFree.argtypes = [ctypes.c_void_p]
    return lib


class Contig:
    """hipExtMallocWithFlags(..., hipDeviceMallocContiguous = 0x4)."""

    def __init__(self, nbytes):
        self.lib = _hip()
        p = ctypes.c_void_p()
        rc = self.lib.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 0x4)
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags contiguous rc={rc}")
        self.ptr = p.value

    def __del__(self):
        self.lib.hipFree(self.ptr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,3,7")
    ap.add_argument("--mib", default="256,512,1024")
    ap.add_argument("--layouts", default="sep,slab,slab+4k,slab+64k,slab+2m4k")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--sets", default="", help="buffer sets to rotate over (comma list; default: >= 2 GiB)")
    ap.add_argument("--ws-mib", default="",
                    help="working sets to rotate over, in MiB (comma list): sets = max(1, ws / ((m + 1) * bucket)), "
                         "at most 64; overrides --sets")
    ap.add_argument("--gate", action="store_true",
                    help="an untimed spin kernel ahead of the start event (bench.py's gate): the host enqueues "
                         "the timed launches while the GPU is busy, so small buckets are not host-bound")
    ap.add_argument("--tag", default="", help="copied into every line (e.g. the A/B arm)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    for m in [int(x) for x in a.ms.split(",")]:
        for mib in [int(x) for x in a.mib.split(",")]:
            nbytes = mib << 20
            n = nbytes // 4
            auto = max(1, min(4, (2048 << 20) // ((m + 1) * nbytes)))
            if a.ws_mib:
                set_list = [max(1, min(64, (int(w) << 20) // ((m + 1) * nbytes))) for w in a.ws_mib.split(",")]
            else:
                set_list = [int(y) for y in a.sets.split(",")] if a.sets else [auto]
            for lay, sets in [(x, y) for x in a.layouts.split(",") for y in set_list]:
                bufs, keep = [], []
                for si in range(sets):
                    if lay.split("/")[0] == "contig":
                        ops = [Contig(nbytes) for _ in range(m + 1)]
                        keep.append(ops)
                        ptrs = [o.ptr for o in ops]
                    elif lay.split("/")[0] == "sep":
                        ops = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(m + 1)]
                        keep.append(ops)
                        ptrs = [t.data_ptr() for t in ops]
                    else:
                        d = DELTAS[lay]
                        slab = torch.empty((m + 1) * (nbytes + d) + 4096, dtype=torch.uint8, device=dev)
                        keep.append(slab)
                        ptrs = [slab.data_ptr() + j * (nbytes + d) for j in range(m + 1)]
                    for j, p in enumerate(ptrs):
                        ca.check(ca.fill(p, n, ca.FLOAT32, 0, 3, 16 * si + j, stream=s))
                    bufs.append(ptrs)
                torch.cuda.synchronize()

                split = int(lay.split("/s")[1]) if "/s" in lay else 1
                piece = ((n + split - 1) // split + 255) // 256 * 256

                def go(i):
                    p = bufs[i % sets]
                    rc = 0
                    for o in range(0, n, piece):
                        c = min(piece, n - o)
                        rc = rc or ca.reduce_multi(p[0] + 4 * o, p[0] + 4 * o, [q + 4 * o for q in p[1:]], c,
                                                   ca.FLOAT32, ca.SUM, s)
                    return rc

                for i in range(2):
                    ca.check(go(i))
                for i in range(sets):  # every set streamed once before timing
                    ca.check(go(i))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                if a.gate:
                    torch.cuda._sleep(1_000_000)
                e0.record(s)
                for i in range(a.reps):
                    go(i)
                e1.record(s)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.reps * 1e3
                gbps = (m + 2) * nbytes / (us * 1e-6) / 1e9
                print(json.dumps({"m": m, "bucket_MiB": mib, "layout": lay, "sets": sets,
                                  "working_set_MiB": sets * (m + 1) * mib, "tag": a.tag,
                                  "nt": os.environ.get("CHR_REDUCE_NT", "policy"), "reps": a.reps, "us": round(us, 2),
                                  "GBps": round(gbps, 1), "frac": round(gbps / 8000, 4)}), flush=True)
                del bufs, keep
                torch.cuda.synchronize()
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
