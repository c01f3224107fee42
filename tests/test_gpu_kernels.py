"""HIP bucket-reduction kernels vs the oracle's MPI_Reduce_local restatement.

Bar: bit-exact for every dtype (f32/f64 IEEE with the reference's association, int32
wrapping, bf16 per-step RNE) -- the kernels restate the same per-element operations."""
import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po

pytestmark = pytest.mark.gpu

DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32, "bf16": ca.BFLOAT16, "i8": ca.INT8, "u8": ca.UINT8,
      "i16": ca.INT16, "u16": ca.UINT16, "u32": ca.UINT32, "i64": ca.INT64, "u64": ca.UINT64,
      "fi": ca.FLOAT_INT, "di": ca.DOUBLE_INT, "li": ca.LONG_INT, "2i": ca.TWO_INT, "si": ca.SHORT_INT,
      "cf": ca.C_FLOAT_COMPLEX, "cd": ca.C_DOUBLE_COMPLEX}
OP = {"sum": ca.SUM, "prod": ca.PROD, "max": ca.MAX, "min": ca.MIN, "land": ca.LAND, "lor": ca.LOR,
      "lxor": ca.LXOR, "band": ca.BAND, "bor": ca.BOR, "bxor": ca.BXOR, "maxloc": ca.MAXLOC, "minloc": ca.MINLOC}
INT_OPS = ("sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor")


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


def _bits(a):
    """Raw element bits (structured pair / complex elements: their bytes, padding included)."""
    if a.dtype.names is not None or a.itemsize == 16:
        return a.view(np.uint8)
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


def _bytes_copy(a):
    """A copy that keeps padding bytes (a structured array's .copy() does not)."""
    return a.view(np.uint8).copy().view(a.dtype)


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
    ref = po.reduce_multi(_bytes_copy(acc), ins, dtype, op)
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
    """>= 40 MiB calls switch to the non-temporal one-wave instantiation."""
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
    """Calls that stream >= 40 MiB take the nt / one-wave / ACC0 instantiation: ragged counts and
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


@pytest.mark.parametrize("dtype", ["fi", "di", "li", "2i", "si"])
@pytest.mark.parametrize("op", ["maxloc", "minloc"])
@pytest.mark.parametrize("m", [1, 3, 8, 9])
def test_pair_types_maxloc_minloc(gu, dtype, op, m):
    """MPI_MAXLOC / MPI_MINLOC on MPI's five pair types (MPICH's loop: equal values keep inout's
    value with the lower index, a better incoming element replaces the whole element, NaN compares
    keep inout): vector path (2 or 1 elements per 16-B vector), a ragged tail, a misaligned scalar
    path; the floating pairs also on the TIES pattern (-0 / +0, NaN payloads)."""
    pats = [po.PAT_UNIFORM] + ([po.PAT_TIES] if dtype in ("fi", "di") else [])
    for pat in pats:
        _check_multi(gu, dtype, op, m, 30011, pattern=pat)
        _check_multi(gu, dtype, op, m, 501, off=1, in_off=1, pattern=pat)
        _check_multi(gu, dtype, op, m, 377, off=1, in_off=2, pattern=pat)


@pytest.mark.parametrize("dtype", ["cf", "cd"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("m", [1, 2, 8, 9])
def test_complex_types_sum_prod(gu, dtype, op, m):
    """MPI_SUM / MPI_PROD on MPI_C_FLOAT_COMPLEX / MPI_C_DOUBLE_COMPLEX (C99 complex arithmetic, the
    products rounded one by one): bit-exact on finite data."""
    _check_multi(gu, dtype, op, m, 20011)
    _check_multi(gu, dtype, op, m, 333, off=1, in_off=2)


def test_complex_prod_special_values_match_mpich_fixture(gu):
    """C99 Annex G multiplication (infinities recovered where the plain formula gives NaN + NaN i)
    on MPICH's own fixture inputs (tests/golden/pairs_reduce_local.npz): the device result equals
    MPICH's, NaN parts compared by NaN-ness (the sign / payload of an invalid operation's NaN is the
    x86 default NaN on the CPU, not pinned by C)."""
    import os

    from test_pairs_oracle import complex_equal

    fix = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pairs_reduce_local.npz"))
    for dtype, npdt in (("cf", np.complex64), ("cd", np.complex128)):
        for op in ("sum", "prod"):
            x = fix[f"{dtype}_{op}_in"].copy()
            y = fix[f"{dtype}_{op}_inout"].copy()
            d_x, d_y = gu.to_dev(x), gu.to_dev(y)
            assert ca.reduce_local(d_x, d_y, x.size // np.dtype(npdt).itemsize, DT[dtype], OP[op], gu.stream()) == 0
            gu.sync()
            assert complex_equal(gu.from_dev(d_y, npdt), fix[f"{dtype}_{op}_out"].view(npdt)), (dtype, op)


def test_pair_fixture_bit_exact_on_device(gu):
    """MAXLOC / MINLOC on MPICH's own fixture inputs (integer extremes, ties, -0 / +0, infinities, NaN
    payloads, padding bytes set to a marker): the device result equals MPICH's byte for byte."""
    import os

    fix = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pairs_reduce_local.npz"))
    for dtype in po.PAIR_DTYPES:
        for op in ("maxloc", "minloc"):
            x = fix[f"{dtype}_{op}_in"].copy()
            y = fix[f"{dtype}_{op}_inout"].copy()
            d_x, d_y = gu.to_dev(x), gu.to_dev(y)
            n = x.size // po.NP_DTYPES[dtype].itemsize
            assert ca.reduce_local(d_x, d_y, n, DT[dtype], OP[op], gu.stream()) == 0
            gu.sync()
            got = d_y.cpu().numpy()
            assert np.array_equal(got, fix[f"{dtype}_{op}_out"]), (dtype, op)


@pytest.mark.parametrize("dtype", ["fi", "di"])
def test_pair_running_first_order(gu, dtype):
    """chr_reduce_multi_ex(CHR_REDUCE_RUNNING_FIRST) on the floating pairs: MPICH_do_reduce's order,
    MPI_Reduce_local(running, next) per step, differs bitwise from the default on ties (-0 / +0) and
    NaN compares; checked against the oracle chained the same way."""
    npdt = po.NP_DTYPES[dtype]
    n, m = 20011, 5
    acc = po.fill(n, dtype, po.PAT_TIES, 9, 0)
    ins = [po.fill(n, dtype, po.PAT_TIES, 9, r + 1) for r in range(m)]
    for op in ("maxloc", "minloc"):
        run = _bytes_copy(acc)
        for x in ins:
            nxt = _bytes_copy(x)
            po.reduce_local(run, nxt, dtype, op)  # MPI_Reduce_local(in = running, inout = next)
            run = nxt
        d_acc = gu.to_dev(acc)
        d_ins = [gu.to_dev(x) for x in ins]
        rc = ca.reduce_multi_ex(d_acc, d_acc, d_ins, n, DT[dtype], OP[op], ca.REDUCE_RUNNING_FIRST, gu.stream())
        assert rc == 0
        gu.sync()
        assert np.array_equal(gu.from_dev(d_acc, npdt).view(np.uint8), run.view(np.uint8)), (dtype, op)
        default = po.reduce_multi(_bytes_copy(acc), ins, dtype, op)
        assert not np.array_equal(default.view(np.uint8), run.view(np.uint8))  # the order is visible


def test_pair_and_complex_reject_other_ops(gu):
    x = gu.empty_dev(256)
    for dt in (ca.FLOAT_INT, ca.DOUBLE_INT, ca.LONG_INT, ca.TWO_INT, ca.SHORT_INT):
        for op in (ca.SUM, ca.PROD, ca.MAX, ca.MIN, ca.LAND, ca.BAND):
            assert ca.reduce_local(x, x, 4, dt, op, gu.stream()) == 1
    for dt in (ca.C_FLOAT_COMPLEX, ca.C_DOUBLE_COMPLEX):
        for op in (ca.MAX, ca.MIN, ca.LAND, ca.BXOR, ca.MAXLOC):
            assert ca.reduce_local(x, x, 4, dt, op, gu.stream()) == 1
    for dt in (ca.FLOAT32, ca.INT32, ca.BFLOAT16):
        assert ca.reduce_local(x, x, 4, dt, ca.MAXLOC, gu.stream()) == 1
