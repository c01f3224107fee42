"""NaN payloads through SUM and PROD: which operand's NaN survives when two meet.

IEEE 754 leaves the payload of an operation on two NaNs to the implementation.  The reference's arithmetic is MPICH's C
loop `inout[i] = in[i] + inout[i]` on x86, where the running value's (inout's) NaN survives, quieted;
the oracle restates that loop and gives the same (checked below on CPU values).  On gfx950 the NaN that survives
is the first source operand's, and the compiler is free to commute an add or a multiply, so the kernels' operand
order is what decides: these cases pin it.  Every element of every operand is a NaN with its own payload (and a
second set mixes NaNs with numbers), through the bucket kernel (plain and streaming shapes) and the tree kernel
(the compile-time programs and the run-time interpreter), against the oracle, bit for bit."""
import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po
from tree_util import tree_ref

DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "bf16": ca.BFLOAT16}
OP = {"sum": ca.SUM, "prod": ca.PROD}
NAN_BITS = {"f32": (np.uint32, 0x7F800000, 23), "f64": (np.uint64, 0x7FF0000000000000, 52), "bf16": (np.uint16, 0x7F80, 7)}


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


def _nans(n, dtype, operand, mixed, seed=3):
    """n elements: NaNs whose payload encodes (operand, element) -- quiet and signalling, either sign -- or, when
    `mixed`, every third element a small number instead."""
    udt, exp, mbits = NAN_BITS[dtype]
    rng = np.random.default_rng(seed + 101 * operand)
    pay = (rng.integers(1, 1 << min(mbits, 20), n, dtype=np.uint64) | np.uint64(1)) & np.uint64((1 << mbits) - 1)
    sign = rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(NAN_BITS[dtype][0](0).itemsize * 8 - 1)
    bits = (np.uint64(exp) | pay | sign).astype(udt)
    a = bits.view(po.NP_DTYPES[dtype]) if dtype != "bf16" else bits
    if mixed:
        num = po.fill(n, dtype, 0, seed, operand)
        a = a.copy()
        a[::3] = num[::3]
    return a


def _bits(a):
    return a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


@pytest.mark.parametrize("dtype, ins, inouts, want", [
    ("f32", [0x7FC00001, 0x7F800002, 0xFFC00003, 0x3F800000], [0x7FC00100, 0x7FC00200, 0x7F800300, 0x7F800400],
     [0x7FC00100, 0x7FC00200, 0x7FC00300, 0x7FC00400]),
    ("f64", [0x7FF8000000000001, 0x7FF0000000000002, 0x3FF0000000000000],
     [0x7FF8000000000100, 0x7FF0000000000200, 0xFFF0000000000300],
     [0x7FF8000000000100, 0x7FF8000000000200, 0xFFF8000000000300]),
    ("bf16", [0x7FC1, 0x7F82, 0xFFC3, 0x3F80], [0x7FD0, 0x7FE0, 0x7F90, 0x7F91], [0x7FD0, 0x7FE0, 0x7FD0, 0x7FD1]),
])
def test_oracle_keeps_the_running_values_nan(dtype, ins, inouts, want):
    """The x86 rule the reference's C loop follows for float and double, as the oracle restates it (and writes out
    for bf16, the build's own type): inout's NaN survives, quieted; a lone NaN survives whichever side it is on."""
    udt = NAN_BITS[dtype][0]
    view = (lambda a: a) if dtype == "bf16" else (lambda a: a.view(po.NP_DTYPES[dtype]))
    for op in ("sum", "prod"):
        r = view(np.array(inouts, dtype=udt))
        po.reduce_local(view(np.array(ins, dtype=udt)), r, dtype, op)
        assert [int(x) for x in r.view(udt)] == want


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("m", [1, 3, 7])
@pytest.mark.parametrize("n, mixed", [(50021, False), (50021, True), (6 << 20, False)])
def test_bucket_kernel_nan_payloads(gu, dtype, op, m, n, mixed):
    """chr_reduce_multi: the plain shape, and from 40 MiB per call the streaming one (6 Mi elements x (m + 2))."""
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    if (m + 2) * n * es < (40 << 20) and n > 100000:
        n = (40 << 20) // ((m + 2) * es) + 4099
    acc = _nans(n, dtype, 0, mixed)
    ins = [_nans(n, dtype, j + 1, mixed) for j in range(m)]
    d_acc = gu.to_dev(acc)
    d_ins = [gu.to_dev(x) for x in ins]
    assert ca.reduce_multi(d_acc.data_ptr(), d_acc.data_ptr(), [t.data_ptr() for t in d_ins], n, DT[dtype], OP[op],
                           gu.stream()) == 0
    gu.sync()
    ref = acc.copy()
    for x in ins:
        po.reduce_local(x, ref, dtype, op)
    np.testing.assert_array_equal(_bits(gu.from_dev(d_acc, npdt)), _bits(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("m, n, off", [(3, 50021, 0), (3, 777, 1), (1, 6 << 20, 0)])
def test_bucket_kernel_nan_payloads_running_first_and_misaligned(gu, dtype, op, m, n, off):
    """CHR_REDUCE_RUNNING_FIRST (MPICH_do_reduce's order: every step MPI_Reduce_local(running, next), so the
    incoming operand is inout and its NaN survives), on the vector shapes and, one element off the 16-B grid, on
    the scalar kernel; and the default order on the scalar kernel."""
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    if (m + 2) * n * es < (40 << 20) and n > 100000:
        n = (40 << 20) // ((m + 2) * es) + 4099
    acc = _nans(n, dtype, 0, True)
    ins = [_nans(n, dtype, j + 1, True) for j in range(m)]
    for flags in (ca.REDUCE_RUNNING_FIRST, 0):
        d_acc = gu.empty_dev((n + off) * es)
        d_acc[off * es:(off + n) * es] = gu.to_dev(acc)
        d_ins = []
        for x in ins:
            t = gu.empty_dev((n + 2 * off) * es)  # a different misalignment from the accumulator's
            t[2 * off * es:(2 * off + n) * es] = gu.to_dev(x)
            d_ins.append(t)
        assert ca.reduce_multi_ex(d_acc.data_ptr() + off * es, d_acc.data_ptr() + off * es,
                                  [t.data_ptr() + 2 * off * es for t in d_ins], n, DT[dtype], OP[op], flags,
                                  gu.stream()) == 0
        gu.sync()
        ref = acc.copy()
        for x in ins:
            if flags:
                nxt = x.copy()
                po.reduce_local(ref, nxt, dtype, op)
                ref = nxt
            else:
                po.reduce_local(x, ref, dtype, op)
        np.testing.assert_array_equal(_bits(gu.from_dev(d_acc, npdt)[off:off + n]), _bits(ref))


C4_TREE = ([0, 1, 1, 1, 0, 1, 1, 2], [0] * 7)        # a compile-time program (reduce_tree.hpp StaticProgs<8>)
B2_TREE = ([0, 1, 0, 2, 0, 2, 0, 2], [0] * 7)        # another
ODD_TREE = ([0, 0, 1, 1, 0, 1, 1, 3], [0] * 7)       # not in the table: the run-time interpreter
SWAP_TREE = ([0, 1, 1, 1, 0, 1, 1, 2], [1, 0, 1, 0, 1, 0, 1])  # swapped combines: the interpreter


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16"])
@pytest.mark.parametrize("op", ["sum", "prod"])
@pytest.mark.parametrize("prog", [C4_TREE, B2_TREE, ODD_TREE, SWAP_TREE], ids=["c4", "b2", "interp", "swap"])
@pytest.mark.parametrize("n, mixed", [(40009, False), (40009, True), (2 << 20, False)])
def test_tree_kernel_nan_payloads(gu, dtype, op, prog, n, mixed):
    """chr_reduce_tree, 8 leaves: the plain shape, and from 64 MiB per launch the streaming one."""
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    if 9 * n * es < (64 << 20) and n > 100000:
        n = (64 << 20) // (9 * es) + 4099
    comb, swaps = prog
    leaves = [_nans(n, dtype, j, mixed) for j in range(8)]
    d = [gu.to_dev(x) for x in leaves]
    out = gu.empty_dev(n * es)
    assert ca.reduce_tree(out.data_ptr(), [t.data_ptr() for t in d], comb, swaps, n, DT[dtype], OP[op],
                          gu.stream()) == 0
    gu.sync()
    np.testing.assert_array_equal(_bits(gu.from_dev(out, npdt)), _bits(tree_ref(leaves, comb, swaps, dtype, op)))


# ---- MPICH's own NaN results (tests/golden/nan_reduce_local.npz, tests/golden/gen_nan_payloads.py) ------------------
# Two-NaN, one-NaN and invalid operations (inf - inf, 0 * inf: x86's default NaN, sign set) on every floating type x
# op -- MPI_FLOAT / MPI_DOUBLE SUM and PROD, the C complex types' SUM and PROD in both parts (libgcc's __mulsc3
# included), MPI_FLOAT_INT / MPI_DOUBLE_INT MAXLOC and MINLOC -- as MPICH 3.3.2's MPI_Reduce_local computed them.
NAN_CASES = [("f32", "sum"), ("f32", "prod"), ("f64", "sum"), ("f64", "prod"), ("cf", "sum"), ("cf", "prod"),
             ("cd", "sum"), ("cd", "prod"), ("fi", "maxloc"), ("fi", "minloc"), ("di", "maxloc"), ("di", "minloc")]
NAN_DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "cf": ca.C_FLOAT_COMPLEX, "cd": ca.C_DOUBLE_COMPLEX,
          "fi": ca.FLOAT_INT, "di": ca.DOUBLE_INT}
NAN_OP = {"sum": ca.SUM, "prod": ca.PROD, "maxloc": ca.MAXLOC, "minloc": ca.MINLOC}


@pytest.fixture(scope="module")
def nan_fix():
    import os

    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "nan_reduce_local.npz"),
                   allow_pickle=False)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype, op", NAN_CASES, ids=[f"{d}_{o}" for d, o in NAN_CASES])
def test_mpich_nan_fixture_on_device(gu, nan_fix, dtype, op):
    """MPICH's bytes, element for element, through every kernel shape that can run the (type, op): the scalar kernel
    (chr_reduce_local), the vector kernel plain and -- for f32 / f64, tiled to 48 / 96 MiB per call -- streaming,
    MPICH_do_reduce's running-value-first order (chr_reduce_multi_ex with the operands exchanged), and the tree
    kernel's 2-leaf program, plain and swapped."""
    key = f"{dtype}_{op}"
    x, y, want = nan_fix[key + "_in"], nan_fix[key + "_inout"], nan_fix[key + "_out"]
    ext = po.NP_DTYPES[dtype].itemsize if dtype in ("fi", "di") else np.dtype(po.NP_DTYPES[dtype]).itemsize
    n = x.size // ext
    dt, o = NAN_DT[dtype], NAN_OP[op]
    # scalar kernel: MPI_Reduce_local(in, inout) one element off the 16-B grid
    d_x, d_y = gu.empty_dev(x.size + ext), gu.empty_dev(y.size + ext)
    d_x[ext:] = gu.to_dev(x)
    d_y[ext:] = gu.to_dev(y)
    assert ca.reduce_local(d_x.data_ptr() + ext, d_y.data_ptr() + ext, n, dt, o, gu.stream()) == 0
    gu.sync()
    assert np.array_equal(d_y.cpu().numpy()[ext:], want), "scalar"
    reps = 1024 if dtype in ("f32", "f64") else 4
    xs, ys, ws = np.tile(x, reps), np.tile(y, reps), np.tile(want, reps)
    N = n * reps
    # vector kernel, m = 1 (plain, or streaming from 40 MiB per call)
    d_x, d_y, d_o = gu.to_dev(xs), gu.to_dev(ys), gu.empty_dev(ys.size)
    assert ca.reduce_multi(d_o.data_ptr(), d_y.data_ptr(), [d_x.data_ptr()], N, dt, o, gu.stream()) == 0
    gu.sync()
    assert np.array_equal(d_o.cpu().numpy(), ws), "vector"
    # running-value-first: MPI_Reduce_local(in = running, inout = next), the running value being the accumulator
    assert ca.reduce_multi_ex(d_o.data_ptr(), d_x.data_ptr(), [d_y.data_ptr()], N, dt, o, ca.REDUCE_RUNNING_FIRST,
                              gu.stream()) == 0
    gu.sync()
    assert np.array_equal(d_o.cpu().numpy(), ws), "running first"
    # tree kernel, 2 leaves: F(in = leaf 1, inout = leaf 0); swapped: F(in = leaf 0, inout = leaf 1)
    for leaves, swaps in (([d_y, d_x], [0]), ([d_x, d_y], [1])):
        assert ca.reduce_tree(d_o.data_ptr(), [t.data_ptr() for t in leaves], [0, 1], swaps, N, dt, o,
                              gu.stream()) == 0
        gu.sync()
        assert np.array_equal(d_o.cpu().numpy(), ws), ("tree", swaps)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype, op", NAN_CASES, ids=[f"{d}_{o}" for d, o in NAN_CASES])
def test_nan_fixture_chains_vs_oracle(gu, nan_fix, dtype, op):
    """Chains of the fixture's NaN-rich operands: m = 3 fused folds and an 8-leaf tree (a compile-time program and a
    swapped one), against the oracle, whose single steps the fixture pins."""
    key = f"{dtype}_{op}"
    npdt = po.NP_DTYPES[dtype]
    raw = [nan_fix[key + "_in"], nan_fix[key + "_inout"], nan_fix[key + "_out"]]
    ext = npdt.itemsize if dtype in ("fi", "di") else np.dtype(npdt).itemsize
    n = raw[0].size // ext
    rng = np.random.default_rng(7)
    ops = [np.ascontiguousarray(raw[j % 3].reshape(n, ext)[rng.permutation(n)]).reshape(-1) for j in range(8)]
    dt, o = NAN_DT[dtype], NAN_OP[op]
    d = [gu.to_dev(a) for a in ops]
    out = gu.empty_dev(ops[0].size)
    assert ca.reduce_multi(out.data_ptr(), d[0].data_ptr(), [t.data_ptr() for t in d[1:4]], n, dt, o, gu.stream()) == 0
    gu.sync()
    ref = ops[0].copy().view(npdt)
    for a in ops[1:4]:
        po.reduce_local(a.copy().view(npdt), ref, dtype, op)
    assert np.array_equal(out.cpu().numpy(), ref.view(np.uint8)), "m = 3"
    for comb, swaps in (C4_TREE, SWAP_TREE):
        assert ca.reduce_tree(out.data_ptr(), [t.data_ptr() for t in d], comb, swaps, n, dt, o, gu.stream()) == 0
        gu.sync()
        want = tree_ref([a.copy().view(npdt) for a in ops], comb, swaps, dtype, op)
        assert np.array_equal(out.cpu().numpy(), want.view(np.uint8)), ("tree", swaps)
