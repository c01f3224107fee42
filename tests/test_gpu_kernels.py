"""HIP bucket-reduction kernels vs the oracle's MPI_Reduce_local restatement.

Bar: bit-exact for every dtype (f32/f64 IEEE with the reference's association, int32
wrapping, bf16 per-step RNE) -- the kernels restate the same per-element operations."""
import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po

pytestmark = pytest.mark.gpu

DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32, "bf16": ca.BFLOAT16, "i8": ca.INT8, "u8": ca.UINT8,
      "i16": ca.INT16, "u16": ca.UINT16, "u32": ca.UINT32, "i64": ca.INT64, "u64": ca.UINT64}
OP = {"sum": ca.SUM, "prod": ca.PROD, "max": ca.MAX, "min": ca.MIN, "land": ca.LAND, "lor": ca.LOR,
      "lxor": ca.LXOR, "band": ca.BAND, "bor": ca.BOR, "bxor": ca.BXOR}
INT_OPS = ("sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor")


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


def _bits(a):
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


def _check_multi(gu, dtype, op, m, n, off=0, in_off=None, seed=5, pattern=0):
    """out = acc op ins[0] ... op ins[m-1] on device, element offsets to test alignment."""
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    in_off = off if in_off is None else in_off
    acc = po.fill(n, dtype, pattern, seed, 0)
    ins = [po.fill(n, dtype, pattern, seed, r + 1) for r in range(m)]
    if op == "prod" and dtype == "i32":
        ins = [(x % 7).astype(np.int32) for x in ins]
    d_acc = gu.empty_dev((n + off) * es)
    d_acc[off * es:(off + n) * es] = gu.to_dev(acc)
    d_ins = []
    for x in ins:
        t = gu.empty_dev((n + in_off) * es)
        t[in_off * es:(in_off + n) * es] = gu.to_dev(x)
        d_ins.append(t)
    rc = ca.reduce_multi(d_acc.data_ptr() + off * es, d_acc.data_ptr() + off * es,
                         [t.data_ptr() + in_off * es for t in d_ins], n, DT[dtype], OP[op], gu.stream())
    assert rc == 0
    gu.sync()
    got = gu.from_dev(d_acc, npdt)[off:off + n]
    ref = po.reduce_multi(acc.copy(), ins, dtype, op)
    np.testing.assert_array_equal(_bits(got), _bits(ref))


@pytest.mark.parametrize("dtype", ["f32", "f64", "i32", "bf16"])
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min"])
@pytest.mark.parametrize("m", [1, 3, 7])
def test_reduce_multi_all_dtypes_ops(gu, dtype, op, m):
    _check_multi(gu, dtype, op, m, 100003)


@pytest.mark.parametrize("m", [1, 2, 4, 5, 6, 8, 9, 16, 17])
def test_fan_in_and_chaining(gu, m):
    _check_multi(gu, "f32", "sum", m, 65536 + 13)
    _check_multi(gu, "bf16", "sum", m, 4099)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 7, 8, 9, 255, 256, 1023, 1024, 1025, 4096 * 4 + 3])
def test_edge_sizes(gu, n):
    for dt in ("f32", "bf16", "f64"):
        _check_multi(gu, dt, "sum", 3, n)


@pytest.mark.parametrize("off,in_off", [(1, 1), (3, 3), (2, 2), (1, 2), (0, 3), (5, 0)])
def test_misaligned_buffers(gu, off, in_off):
    for dt in ("f32", "bf16", "i32"):
        _check_multi(gu, dt, "sum", 2, 10007, off, in_off)


@pytest.mark.parametrize("dtype", ["i8", "u8", "i16", "u16", "i32", "u32", "i64", "u64"])
@pytest.mark.parametrize("op", INT_OPS)
@pytest.mark.parametrize("m", [1, 3, 8, 9])
def test_integer_types_and_logical_bitwise_ops(gu, dtype, op, m):
    """MPI integer types beyond int32 and LAND/LOR/LXOR/BAND/BOR/BXOR (the reference's generic
    MPI_Datatype x MPI_Op, all_reduce_radix_batch.cpp:202-204): vector path, a ragged tail, a
    misaligned scalar path; the logical ops on the SPARSE / TIES patterns so both results occur."""
    pat = {"land": po.PAT_SPARSE, "lor": po.PAT_TIES, "lxor": po.PAT_TIES}.get(op, po.PAT_UNIFORM)
    _check_multi(gu, dtype, op, m, 50021, pattern=pat)
    _check_multi(gu, dtype, op, m, 999, off=1, in_off=1, pattern=pat)
    _check_multi(gu, dtype, op, m, 777, off=1, in_off=2, pattern=pat)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("op", ["land", "lor", "lxor"])
@pytest.mark.parametrize("m", [1, 4])
def test_float_logical_ops(gu, dtype, op, m):
    """MPICH 3.3.2 accepts LAND/LOR/LXOR on float and double (C truth: NaN true, -0 false): ties
    data (+-0, +-1, 0.5, NaN payloads)."""
    _check_multi(gu, dtype, op, m, 30011, pattern=po.PAT_TIES)
    _check_multi(gu, dtype, op, m, 501, off=1, in_off=1, pattern=po.PAT_TIES)


@pytest.mark.parametrize("dtype", ["u8", "i16", "i64", "u64"])
def test_integer_types_streaming_path(gu, dtype):
    """>= 128 MiB calls switch to the non-temporal one-wave instantiation."""
    n = (48 << 20) // np.dtype(po.NP_DTYPES[dtype]).itemsize
    _check_multi(gu, dtype, "sum", 1, n)
    _check_multi(gu, dtype, "max", 3, n // 2 + 7)


def test_float_types_reject_bitwise_ops(gu):
    x = gu.empty_dev(64)
    for dt in (ca.FLOAT32, ca.FLOAT64, ca.BFLOAT16):
        for op in (ca.BAND, ca.BOR, ca.BXOR):
            assert ca.reduce_local(x, x, 4, dt, op, gu.stream()) == 1
    for op in (ca.LAND, ca.LOR, ca.LXOR):  # bf16 is this library's own type: arithmetic and MAX/MIN
        assert ca.reduce_local(x, x, 4, ca.BFLOAT16, op, gu.stream()) == 1
    assert ca.reduce_local(x, x, 4, 11, ca.SUM, gu.stream()) == 1
    assert ca.reduce_local(x, x, 4, ca.INT8, 10, gu.stream()) == 1


def test_reduce_local_mpi_semantics(gu):
    """MPI_Reduce_local (MPICH loop): inout = OP(inout, in); MAX keeps inout only when
    inout > in, so ties (-0/+0) and NaN compares take `in`."""
    a = np.array([1.0, -0.0, np.nan, 3.0, 0.0, -np.inf], dtype=np.float32)
    b = np.array([2.0, 0.0, 1.0, np.nan, -0.0, np.inf], dtype=np.float32)
    for op in ("max", "min", "sum", "prod"):
        da, db = gu.to_dev(a), gu.to_dev(b)
        assert ca.reduce_local(da, db, a.size, ca.FLOAT32, OP[op], gu.stream()) == 0
        gu.sync()
        ref = po.reduce_local(a, b.copy(), "f32", op)
        np.testing.assert_array_equal(_bits(gu.from_dev(db, np.float32)), _bits(ref))
    # bf16 NaN payloads and RNE ties
    x = np.array([0x7FC1, 0x3F80, 0x3F81, 0xFF80, 0x0001], dtype=np.uint16)
    y = np.array([0x3F80, 0x3B80, 0x3B80, 0x7F80, 0x8001], dtype=np.uint16)
    dx, dy = gu.to_dev(x), gu.to_dev(y)
    assert ca.reduce_local(dx, dy, x.size, ca.BFLOAT16, ca.SUM, gu.stream()) == 0
    gu.sync()
    np.testing.assert_array_equal(gu.from_dev(dy, np.uint16), po.reduce_local(x, y.copy(), "bf16", "sum"))


def test_int32_wraps(gu):
    a = np.array([2**31 - 1, -(2**31), 123], dtype=np.int32)
    b = np.array([1, -1, -123], dtype=np.int32)
    da, db = gu.to_dev(a), gu.to_dev(b)
    assert ca.reduce_local(da, db, 3, ca.INT32, ca.SUM, gu.stream()) == 0
    gu.sync()
    assert list(gu.from_dev(db, np.int32)) == [-(2**31), 2**31 - 1, 0]


@pytest.mark.parametrize("dtype", ["f32", "f64", "i32", "bf16", "i8", "u8", "i16", "u16", "u32", "i64", "u64"])
@pytest.mark.parametrize("pattern", [0, 1, 2, 3])
def test_device_fill_matches_oracle_generator(gu, dtype, pattern):
    n = 300001
    npdt = po.NP_DTYPES[dtype]
    d = gu.empty_dev(n * np.dtype(npdt).itemsize)
    assert ca.fill(d, n, DT[dtype], pattern, 0xC41A5EED, 5, stream=gu.stream()) == 0
    gu.sync()
    np.testing.assert_array_equal(_bits(gu.from_dev(d, npdt)), _bits(po.fill(n, dtype, pattern, 0xC41A5EED, 5)))


@pytest.mark.parametrize("nbytes", [1 << 10, 1 << 20, 64 << 20, 1 << 30])
def test_bucket_sizes_1k_to_1g(gu, nbytes):
    """BASELINE sweep range (1 KiB .. 1 GiB per bucket), k=2 (m=1) and k=4 (m=3): bit-exact."""
    n = nbytes // 4
    _check_multi(gu, "f32", "sum", 1, n, seed=11)
    if nbytes <= 64 << 20:
        _check_multi(gu, "f32", "sum", 3, n, seed=12)


@pytest.mark.parametrize("dtype,op,m,nbytes,off", [("f32", "sum", 1, 64 << 20, 1), ("bf16", "max", 3, 48 << 20, 0),
                                                    ("f64", "sum", 7, 16 << 20, 3), ("i32", "prod", 2, 48 << 20, 2),
                                                    ("bf16", "sum", 1, 64 << 20, 5)])
def test_streaming_path_ragged(gu, dtype, op, m, nbytes, off):
    """Calls that stream >= 128 MiB take the nt / one-wave / ACC0 instantiation: ragged counts and
    misaligned heads there too (scalar head and tail around the vector body)."""
    es = np.dtype(po.NP_DTYPES[dtype]).itemsize
    _check_multi(gu, dtype, op, m, nbytes // es + 12345, off, seed=21)


def test_invalid_args(gu):
    assert ca.reduce_local(0, 0, 0, ca.FLOAT32, ca.SUM) == 0  # n == 0 is a no-op
    assert ca.reduce_local(0, 0, 5, ca.FLOAT32, ca.SUM) == 1
    assert ca.reduce_local(1, 1, 5, 11, ca.SUM) == 1  # 11: no such dtype
    assert ca.reduce_local(1, 1, 5, ca.FLOAT32, 10) == 1  # 10: no such op
    assert ca.reduce_local(1, 1, 5, ca.FLOAT32, ca.BXOR) == 1  # bitwise op on a float type


@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16", "i32"])
@pytest.mark.parametrize("op", ["max", "min", "sum"])
@pytest.mark.parametrize("m", [1, 3, 8, 11])
def test_reduce_multi_running_first(gu, dtype, op, m):
    """CHR_REDUCE_RUNNING_FIRST = MPICH_do_reduce's chain (allreduce_recexch.cpp:147-186):
    every step is MPI_Reduce_local(running, next).  Ties/NaN data make the order visible."""
    n = 4099
    npdt = po.NP_DTYPES[dtype]
    pat = po.PAT_TIES if op != "sum" else po.PAT_UNIFORM
    acc = po.fill(n, dtype, pat, 77, 0)
    ins = [po.fill(n, dtype, pat, 77, j + 1) for j in range(m)]
    run = acc.copy()
    for x in ins:
        nxt = x.copy()
        po.reduce_local(run, nxt, dtype, op)
        run = nxt
    d_acc, d_ins, d_out = gu.to_dev(acc), [gu.to_dev(x) for x in ins], gu.empty_dev(acc.nbytes)
    assert ca.reduce_multi_ex(d_out, d_acc, d_ins, n, DT[dtype], OP[op], ca.REDUCE_RUNNING_FIRST, gu.stream()) == 0
    gu.sync()
    np.testing.assert_array_equal(_bits(gu.from_dev(d_out, npdt)), _bits(run))
    if op != "sum" and dtype != "i32":  # and the default order really differs on this data
        dflt = po.reduce_multi(acc.copy(), ins, dtype, op)
        assert not np.array_equal(_bits(dflt), _bits(run))


def test_reduce_multi_ex_rejects_bad_flags(gu):
    d = gu.empty_dev(64)
    assert ca.reduce_multi_ex(d, d, [d], 4, ca.FLOAT32, ca.MAX, 2, gu.stream()) == 1
