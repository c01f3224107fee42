"""pyoracle -- TEST INFRASTRUCTURE ONLY: ctypes view of oracle/liboracle.so.

The CPU restatement of CHiArA's radix/batch collectives and of MPI_Reduce_local
(see chiara_oracle.h).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

DTYPES = {"f32": 0, "f64": 1, "i32": 2, "bf16": 3, "i8": 4, "u8": 5, "i16": 6, "u16": 7, "u32": 8, "i64": 9,
          "u64": 10, "fi": 11, "di": 12, "li": 13, "2i": 14, "si": 15, "cf": 16, "cd": 17}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "land": 4, "lor": 5, "lxor": 6, "band": 7, "bor": 8, "bxor": 9,
       "maxloc": 10, "minloc": 11,
       "user_halfadd": 12,  # test user op (MPI_Op_create, non-commutative): inout = in * 0.5f + inout, f32
       "user_halfadd_c": 13}  # the same function created commutative (the baselines' commutative paths)
ORC_ERR_OP = 8  # the oracle's MPI_ERR_OP (a baseline refusing a non-commutative op)


def _pair(vfmt, ioff, size):
    return np.dtype({"names": ["v", "i"], "formats": [vfmt, "<i4"], "offsets": [0, ioff], "itemsize": size})


NP_DTYPES = {"f32": np.float32, "f64": np.float64, "i32": np.int32, "bf16": np.uint16, "i8": np.int8, "u8": np.uint8,
             "i16": np.int16, "u16": np.uint16, "u32": np.uint32, "i64": np.int64, "u64": np.uint64,
             # MPI's MAXLOC / MINLOC pair types (C struct layouts) and the C complex types
             "fi": _pair("<f4", 4, 8), "di": _pair("<f8", 8, 16), "li": _pair("<i8", 8, 16), "2i": _pair("<i4", 4, 8),
             "si": _pair("<i2", 4, 8), "cf": np.complex64, "cd": np.complex128}
PAIR_DTYPES = ("fi", "di", "li", "2i", "si")
COMPLEX_DTYPES = ("cf", "cd")


def valid(dtype, op):
    """MPICH 3.3.2's (type, op) table (chiara_oracle.c orc_valid)."""
    lib().orc_valid.restype = ctypes.c_int
    return bool(lib().orc_valid(DTYPES[dtype], OPS[op]))
INT_DTYPES = ("i32", "i8", "u8", "i16", "u16", "u32", "i64", "u64")
PAT_UNIFORM, PAT_SEQ, PAT_TIES, PAT_SPARSE = 0, 1, 2, 3

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        L.orc_fill.argtypes = [vp, sz, i, i, u64, i, u64]
        L.orc_fill_at.argtypes = [vp, sz, i, i, u64, i, u64, u64]
        L.orc_reduce_local.argtypes = [vp, vp, sz, i, i]
        L.orc_reduce_multi.argtypes = [vp, ctypes.POINTER(vp), i, sz, i, i]
        L.orc_allreduce_radix_batch.argtypes = [i, i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.orc_allreduce_radix_batch.restype = i
        L.orc_reduce_scatter_radix_batch.argtypes = [i, i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.orc_reduce_scatter_radix_batch.restype = i
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def fill(n, dtype, pattern, seed, rank, count_for_seq=None):
    """Rank `rank`'s synthetic input (same formula as the golden driver and the device fill)."""
    a = np.empty(n, dtype=NP_DTYPES[dtype])
    lib().orc_fill(_ptr(a), n, DTYPES[dtype], pattern, seed, rank, n if count_for_seq is None else count_for_seq)
    return a


def fill_at(n, dtype, pattern, seed, rank, start, count_for_seq):
    """Elements [start, start + n) of the input fill() makes with this count_for_seq."""
    a = np.empty(n, dtype=NP_DTYPES[dtype])
    lib().orc_fill_at(_ptr(a), n, DTYPES[dtype], pattern, seed, rank, count_for_seq, start)
    return a


def block_window(nblocks, blocklen, off, width):
    """Element indices of the window [off, off + width) of every one of `nblocks` blocks of
    `blocklen` elements, block-major: a (nblocks * width,) index array."""
    return (np.arange(nblocks, dtype=np.int64)[:, None] * blocklen + off + np.arange(width, dtype=np.int64)).ravel()


def window_inputs(nranks, count, off, width, dtype, pattern, seed, nblocks=None):
    """Every rank's input restricted to the block window [off, off + width) of each of its
    `nblocks` (default nranks) blocks of count // nblocks elements.

    Block-window property: all_reduce_radix_batch / reduce_scatter_radix_batch address their
    buffers only in whole blocks of recvcount elements (every offset and count in
    all_reduce_radix_batch.cpp:239-312, :343-364, :523-530 is a multiple of recvcount, IRC =
    recvcount * b), and reduce elementwise, so an element's expression depends only on its block.
    Running the collective on these windows (recvcount' = width) therefore computes, for every
    element, the same expression as the full-size call: the full-size result restricted to the
    window.  tests/test_oracle_golden.py::test_block_window_property pins this on the oracle."""
    nb = nranks if nblocks is None else nblocks
    blen = count // nb
    out = []
    for r in range(nranks):
        parts = [fill_at(width, dtype, pattern, seed, r, j * blen + off, count) for j in range(nb)]
        out.append(np.concatenate(parts))
    return out


def reduce_local(inp, inout, dtype, op):
    """MPI_Reduce_local restated: inout = inp (op) inout, in place."""
    assert inp.size == inout.size
    lib().orc_reduce_local(_ptr(inp), _ptr(inout), inout.size, DTYPES[dtype], OPS[op])
    return inout


def reduce_multi(acc, ins, dtype, op):
    arr = (ctypes.c_void_p * max(1, len(ins)))(*[x.ctypes.data for x in ins])
    lib().orc_reduce_multi(_ptr(acc), arr, len(ins), acc.size, DTYPES[dtype], OPS[op])
    return acc


def _ptr_array(bufs):
    return (ctypes.c_void_p * len(bufs))(*[(b.ctypes.data if b is not None else None) for b in bufs])


def allreduce_radix_batch(sends, k, b, dtype, op, inplace=False):
    """All ranks' outputs of all_reduce_radix_batch.  sends: list (one per rank)."""
    n = len(sends)
    count = sends[0].size
    if inplace:
        recvs = [s.copy() for s in sends]
        sp = _ptr_array([None] * n)
    else:
        recvs = [np.zeros_like(s) for s in sends]
        sp = _ptr_array(sends)
    rc = lib().orc_allreduce_radix_batch(n, k, b, count, DTYPES[dtype], OPS[op], sp, _ptr_array(recvs))
    if rc:
        raise ValueError(f"oracle allreduce rejected geometry (rc={rc})")
    return recvs


def reduce_scatter_radix_batch(sends, k, b, dtype, op, inplace=False):
    n = len(sends)
    recvcount = sends[0].size // n
    if inplace:
        recvs = [s.copy() for s in sends]
        sp = _ptr_array([None] * n)
    else:
        recvs = [np.zeros(recvcount, dtype=s.dtype) for s in sends]
        sp = _ptr_array(sends)
    rc = lib().orc_reduce_scatter_radix_batch(n, k, b, recvcount, DTYPES[dtype], OPS[op], sp, _ptr_array(recvs))
    if rc:
        raise ValueError(f"oracle reduce_scatter rejected geometry (rc={rc})")
    return [r[:recvcount] for r in recvs]


def allgather_radix_batch(sends, k, b, dtype, inplace=False):
    """All ranks' outputs of allgather_radix_batch (n*sendcount each, rank-major)."""
    L = lib()
    if not getattr(L, "_ag_ready", False):
        L.orc_allgather_radix_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                                ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                ctypes.POINTER(ctypes.c_void_p)]
        L.orc_allgather_radix_batch.restype = ctypes.c_int
        L._ag_ready = True
    n = len(sends)
    count = sends[0].size
    recvs = [np.zeros(count * n, dtype=sends[0].dtype) for _ in range(n)]
    if inplace:
        for r in range(n):
            recvs[r][r * count:(r + 1) * count] = sends[r]
    sp = _ptr_array([None] * n) if inplace else _ptr_array(sends)
    rc = L.orc_allgather_radix_batch(n, k, b, count, DTYPES[dtype], sp, _ptr_array(recvs))
    if rc:
        raise ValueError(f"oracle allgather rejected geometry (rc={rc})")
    return recvs


def _setup_mpich(L):
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    for name in ("orc_allreduce_ring", "orc_allreduce_recursive_doubling", "orc_allreduce_reduce_scatter_allgather"):
        fn = getattr(L, name)
        fn.argtypes = [i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        fn.restype = i
    for name in ("orc_allreduce_recexch", "orc_allreduce_recursive_multiplying",
                 "orc_allreduce_k_reduce_scatter_allgather"):
        fn = getattr(L, name)
        fn.argtypes = [i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        fn.restype = i


MPICH_ALGOS = ("ring", "rd", "rsag", "rx", "krsag", "rm")


def mpich_allreduce(algo, sends, dtype, op, k=2, inplace=False):
    """All ranks' outputs of the MPICH baseline `algo` (testing/mpich_implementations/all_reduce/)."""
    L = lib()
    if not getattr(L, "_mpich_ready", False):
        _setup_mpich(L)
        L._mpich_ready = True
    n = len(sends)
    count = sends[0].size
    recvs = [s.copy() for s in sends] if inplace else [np.zeros_like(s) for s in sends]
    sp = _ptr_array([None] * n) if inplace else _ptr_array(sends)
    rp = _ptr_array(recvs)
    if algo == "ring":
        rc = L.orc_allreduce_ring(n, count, DTYPES[dtype], OPS[op], sp, rp)
    elif algo == "rd":
        rc = L.orc_allreduce_recursive_doubling(n, count, DTYPES[dtype], OPS[op], sp, rp)
    elif algo == "rsag":
        rc = L.orc_allreduce_reduce_scatter_allgather(n, count, DTYPES[dtype], OPS[op], sp, rp)
    elif algo == "rx":
        rc = L.orc_allreduce_recexch(n, k, count, DTYPES[dtype], OPS[op], sp, rp)
    elif algo == "rm":
        rc = L.orc_allreduce_recursive_multiplying(n, k, count, DTYPES[dtype], OPS[op], sp, rp)
    elif algo == "krsag":
        rc = L.orc_allreduce_k_reduce_scatter_allgather(n, k, count, DTYPES[dtype], OPS[op], sp, rp)
    else:
        raise ValueError(algo)
    if rc:
        raise ValueError(f"oracle {algo} rejected (rc={rc})", rc)
    return recvs


MPICH_RS_ALGOS = ("rs_radix", "rs_halving", "rs_doubling", "rs_pairwise")


def mpich_reduce_scatter(algo, sends, dtype, op, k=2, inplace=False):
    """All ranks' outputs (recvcount each) of the MPICH baseline reduce-scatter `algo`
    (testing/mpich_implementations/reduce_scatter/).  sends: n*recvcount elements per rank."""
    L = lib()
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    if not getattr(L, "_rs_ready", False):
        for name in ("orc_reduce_scatter_pairwise", "orc_reduce_scatter_rec_halving",
                     "orc_reduce_scatter_rec_doubling"):
            fn = getattr(L, name)
            fn.argtypes = [i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
            fn.restype = i
        L.orc_reduce_scatter_radix.argtypes = [i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.orc_reduce_scatter_radix.restype = i
        L._rs_ready = True
    n = len(sends)
    rc = sends[0].size // n
    recvs = [s.copy() for s in sends] if inplace else [np.zeros(rc, dtype=s.dtype) for s in sends]
    sp = _ptr_array([None] * n) if inplace else _ptr_array(sends)
    rp = _ptr_array(recvs)
    d, o = DTYPES[dtype], OPS[op]
    if algo == "rs_radix":
        rc_ = L.orc_reduce_scatter_radix(n, k, rc, d, o, sp, rp)
    elif algo == "rs_halving":
        rc_ = L.orc_reduce_scatter_rec_halving(n, rc, d, o, sp, rp)
    elif algo == "rs_doubling":
        rc_ = L.orc_reduce_scatter_rec_doubling(n, rc, d, o, sp, rp)
    elif algo == "rs_pairwise":
        rc_ = L.orc_reduce_scatter_pairwise(n, rc, d, o, sp, rp)
    else:
        raise ValueError(algo)
    if rc_:
        raise ValueError(f"oracle {algo} rejected (rc={rc_})", rc_)
    return [r[:rc] for r in recvs]


PHASE_ALGOS = ("irs", "ilr", "isc")  # intra_reduce_scatter_radix / inter_linear_reduce / intra_scatter_radix_batch


def phase_sizes(algo, n, b, rc):
    """(input, output) elements per rank of the stand-alone phase `algo` (testing/custom_implementations/
    work_dir/reduce_scatter/): ranks in n / b groups of b, IRC = rc * b, niters = ceil(nnodes / b)."""
    nnodes = n // b
    niters = nnodes // b + (1 if nnodes % b else 0)
    if algo == "irs":
        return rc * n, niters * rc * b
    if algo == "ilr":
        return niters * rc * b, rc * b
    if algo == "isc":
        return b * rc, rc
    raise ValueError(algo)


def phase_collective(algo, sends, dtype, op, k, b, rc, inplace=False):
    """All ranks' recv buffers (output size, zero where the reference writes nothing) of the stand-alone
    phase `algo`; sends: each rank's input (phase_sizes).  inplace: irs only (MPI_IN_PLACE)."""
    L = lib()
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    if not getattr(L, "_phase_ready", False):
        L.orc_intra_reduce_scatter.argtypes = [i, i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.orc_inter_reduce_linear.argtypes = [i, i, sz, i, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.orc_intra_scatter.argtypes = [i, i, i, sz, i, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        for fn in (L.orc_intra_reduce_scatter, L.orc_inter_reduce_linear, L.orc_intra_scatter):
            fn.restype = i
        L._phase_ready = True
    n = len(sends)
    _, out_n = phase_sizes(algo, n, b, rc)
    npdt = sends[0].dtype
    if inplace:
        assert algo == "irs"
        recvs = [s.copy() for s in sends]
    else:
        recvs = [np.zeros(max(out_n, 1), dtype=npdt) for _ in sends]
    sp = _ptr_array([None] * n) if inplace else _ptr_array(sends)
    rp = _ptr_array(recvs)
    d = DTYPES[dtype]
    if algo == "irs":
        rc_ = L.orc_intra_reduce_scatter(n, k, b, rc, d, OPS[op], sp, rp)
    elif algo == "ilr":
        rc_ = L.orc_inter_reduce_linear(n, b, rc, d, OPS[op], sp, rp)
    else:
        rc_ = L.orc_intra_scatter(n, k, b, rc, d, sp, rp)
    if rc_:
        raise ValueError(f"oracle {algo} rejected (rc={rc_})", rc_)
    return [r[:out_n] for r in recvs]
