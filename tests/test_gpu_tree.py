"""Fused expression-tree kernel (chr_reduce_tree, csrc/reduce_tree.hip) vs the oracle.

The reference op sequence a tree restates is the chain of MPI_Reduce_local calls that
builds one chunk across phases (all_reduce_radix_batch.cpp:332, :364, :446, :529).  The
CPU side evaluates the same post-order program with the oracle's MPI_Reduce_local
restatement, one call per combine.  Bar: bit-exact for every dtype and op, including the
running-value-first (swap) combines and ties/NaN data (pattern 2)."""
import zlib

import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po
from tree_util import random_program, tree_ref

pytestmark = pytest.mark.gpu

DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32, "bf16": ca.BFLOAT16, "i8": ca.INT8, "u8": ca.UINT8,
      "i16": ca.INT16, "u16": ca.UINT16, "u32": ca.UINT32, "i64": ca.INT64, "u64": ca.UINT64,
      "fi": ca.FLOAT_INT, "di": ca.DOUBLE_INT, "li": ca.LONG_INT, "2i": ca.TWO_INT, "si": ca.SHORT_INT,
      "cf": ca.C_FLOAT_COMPLEX, "cd": ca.C_DOUBLE_COMPLEX}
OP = {"sum": ca.SUM, "prod": ca.PROD, "max": ca.MAX, "min": ca.MIN, "land": ca.LAND, "lor": ca.LOR,
      "lxor": ca.LXOR, "band": ca.BAND, "bor": ca.BOR, "bxor": ca.BXOR, "maxloc": ca.MAXLOC, "minloc": ca.MINLOC}


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


def _bits(a):
    if a.dtype.names is not None or a.itemsize == 16:  # pair / complex elements: their bytes
        return a.view(np.uint8)
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


def _run(gu, dtype, op, comb, swaps, n, pattern=0, off=0, seed=11, inplace_leaf=None):
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    nl = len(comb)
    leaves = [po.fill(n, dtype, pattern, seed, r) for r in range(nl)]
    if op == "prod" and dtype == "i32":
        leaves = [(x % 5).astype(np.int32) for x in leaves]
    d = []
    for x in leaves:
        t = gu.empty_dev((n + off) * es)
        t[off * es:(off + n) * es] = gu.to_dev(x)
        d.append(t)
    if inplace_leaf is None:
        out = gu.empty_dev((n + off) * es)
    else:
        out = d[inplace_leaf]
    rc = ca.reduce_tree(out.data_ptr() + off * es, [t.data_ptr() + off * es for t in d], comb, swaps, n,
                        DT[dtype], OP[op], gu.stream())
    assert rc == 0
    gu.sync()
    got = gu.from_dev(out, npdt)[off:off + n]
    ref = tree_ref(leaves, comb, swaps, dtype, op)
    np.testing.assert_array_equal(_bits(got), _bits(ref))


# the shapes the flat schedule emits at the BASELINE geometries (n=8)
C4_TREE = ([0, 1, 1, 1, 0, 1, 1, 2], [0] * 7)       # k=4, b=4: fold4 + fold4, then lane fold
K2B8_TREE = ([0, 1, 0, 2, 0, 1, 0, 3], [0] * 7)     # k=2, b=8: binary recexch, depth 4
K4B8_TREE = ([0, 1, 1, 1, 0, 2, 1, 1], [0] * 7)


@pytest.mark.parametrize("dtype", ["f32", "f64", "i32", "bf16"])
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min"])
@pytest.mark.parametrize("prog", [C4_TREE, K2B8_TREE, K4B8_TREE])
def test_flat_shapes_all_dtypes_ops(gu, dtype, op, prog):
    _run(gu, dtype, op, prog[0], prog[1], 100003, pattern=2 if op in ("max", "min") else 0)


@pytest.mark.parametrize("seed", range(12))
def test_random_programs_with_swaps(gu, seed):
    rng = np.random.default_rng(seed)
    comb, swaps = random_program(rng, int(rng.integers(2, 9)))
    for dtype in ("f32", "bf16"):
        for op in ("sum", "max", "min"):
            _run(gu, dtype, op, comb, swaps, 40000 + seed, pattern=2 if op != "sum" else 0, seed=seed)


@pytest.mark.parametrize("n", [0, 1, 3, 7, 8, 9, 255, 1025, 2 * 256 * 4 * 2 + 5])
def test_edge_sizes(gu, n):
    for dt in ("f32", "bf16", "f64"):
        _run(gu, dt, "sum", *C4_TREE, n)


@pytest.mark.parametrize("off", [1, 2, 3])
def test_misaligned(gu, off):
    for dt in ("f32", "bf16", "i32"):
        _run(gu, dt, "sum", *K2B8_TREE, 10007, off=off)


def test_out_aliases_leaf(gu):
    """MPI_IN_PLACE: the root is written over the rank's own leaf (same element offsets)."""
    for leaf in (0, 3, 7):
        _run(gu, "f32", "sum", *C4_TREE, 70001, inplace_leaf=leaf)


@pytest.mark.parametrize("dtype,op", [("f32", "sum"), ("f32", "max"), ("bf16", "sum"), ("i32", "prod"), ("f64", "min")])
def test_streaming_two_leaf_tree_runs_as_a_fold(gu, dtype, op):
    """A streaming 2-leaf tree is one out-of-place fold on the bucket kernel (reduce_tree.hip): both operand orders
    (swap bit), out separate, out = the running value, and out = the fold's input (kept on the tree kernel), on TIES
    data where the order shows -- bit-exact vs the oracle's tree evaluation."""
    n = (24 << 20) // np.dtype(po.NP_DTYPES[dtype]).itemsize + 5  # 3 x 24 MiB per call: past the 40 MiB threshold
    for swaps in ([0], [1]):
        for leaf in (None, 0, 1):
            _run(gu, dtype, op, [0, 1], swaps, n, pattern=2 if op in ("max", "min") else 0, inplace_leaf=leaf)


def test_large_nt_path(gu):
    """>= 64 MiB streamed per call takes the non-temporal instantiation."""
    _run(gu, "f32", "sum", *C4_TREE, (16 << 20) + 7)


@pytest.mark.parametrize("dtype", ["i8", "u8", "i16", "u16", "i32", "u32", "i64", "u64"])
@pytest.mark.parametrize("op", ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"])
def test_integer_types_and_logical_bitwise_ops(gu, dtype, op):
    """The whole-tree kernel on every MPI integer type and op the reference's generic
    MPI_Datatype x MPI_Op admits (reduce_tree_int.hip), C4's tree and a depth-4 one, plus a
    misaligned (scalar) pass."""
    pat = {"land": po.PAT_SPARSE, "lor": po.PAT_TIES, "lxor": po.PAT_TIES}.get(op, po.PAT_UNIFORM)
    if op == "prod" and dtype == "i32":
        return  # int32 arithmetic is the core instantiation, covered above
    for prog in (C4_TREE, K2B8_TREE):
        _run(gu, dtype, op, prog[0], prog[1], 30011, pattern=pat)
    _run(gu, dtype, op, *K4B8_TREE, 1001, pattern=pat, off=1)


@pytest.mark.parametrize("ntrees,n,off", [(2, 100003, 0), (3, 4097, 1), (8, 2048 + 5, 0), (9, 1000, 0), (2, 0, 0)])
def test_batched_trees_bit_identical(gu, ntrees, n, off):
    """chr_reduce_tree_batch (what the executor does with a slice's chunks): several trees, each with
    its own program, leaves and output, in shared launches (8 segments at most per launch, 9 trees
    = two launches), ragged and misaligned heads/tails on the scalar kernel: every tree equal to
    its own oracle evaluation."""
    rng = np.random.default_rng(ntrees * 7 + n)
    npdt = po.NP_DTYPES["f32"]
    progs = [random_program(rng, 8) for _ in range(ntrees)]
    leaves = [[po.fill(n, "f32", 0, 3, 8 * t + j) for j in range(8)] for t in range(ntrees)]
    d_leaves, outs = [], []
    for t in range(ntrees):
        row = []
        for x in leaves[t]:
            d = gu.empty_dev((n + off) * 4)
            d[off * 4:(off + n) * 4] = gu.to_dev(x)
            row.append(d.data_ptr() + off * 4)
            d_leaves.append(d)
        outs.append(gu.empty_dev((n + off) * 4))
        leaves_ptrs = row
        progs[t] = (progs[t][0], progs[t][1], leaves_ptrs)
    rc = ca.reduce_tree_batch([o.data_ptr() + off * 4 for o in outs], [p[2] for p in progs], [p[0] for p in progs],
                              [p[1] for p in progs], n, ca.FLOAT32, ca.SUM, gu.stream())
    assert rc == 0
    gu.sync()
    for t in range(ntrees):
        got = gu.from_dev(outs[t], npdt)[off:off + n]
        want = tree_ref(leaves[t], progs[t][0], progs[t][1], "f32", "sum")
        np.testing.assert_array_equal(_bits(got), _bits(want))


@pytest.mark.parametrize("dtype,op", [(d, o) for d in ("fi", "di", "li", "2i", "si") for o in ("maxloc", "minloc")] +
                         [(d, o) for d in ("cf", "cd") for o in ("sum", "prod")])
def test_tree_pair_and_complex_types(gu, dtype, op):
    """The fused tree on MPI's pair types (MAXLOC / MINLOC) and the C complex types (SUM / PROD):
    random programs with random swap bits (MPICH_do_reduce order per combine), 2..8 leaves, vector
    path with a ragged tail and the misaligned scalar path; the floating pairs on TIES data, where
    the swap bits change the result bits."""
    rng = np.random.default_rng(zlib.crc32(f"{dtype}-{op}".encode()))
    pat = po.PAT_TIES if dtype in ("fi", "di") else po.PAT_UNIFORM
    for nl in (2, 3, 5, 8):
        comb, swaps = random_program(rng, nl)
        _run(gu, dtype, op, comb, swaps, 4099, pattern=pat)
        _run(gu, dtype, op, comb, swaps, 257, pattern=pat, off=1)
    _run(gu, dtype, op, *C4_TREE, 8192 + 3, pattern=pat, inplace_leaf=0)


def all_programs(nl, max_depth=4):
    """Every valid post-order program with nl leaves and stack depth <= max_depth."""
    out = []

    def rec(j, depth, comb):
        depth += 1
        if depth > max_depth:
            return
        if j == nl - 1:
            out.append(comb + [depth - 1])
            return
        for c in range(0, min(3, depth - 1) + 1):
            rec(j + 1, depth - c, comb + [c])

    rec(0, 0, [])
    return out


@pytest.mark.parametrize("dtype,op", [(d, o) for d in ("fi", "di", "li", "2i", "si") for o in ("maxloc", "minloc")] +
                         [(d, o) for d in ("cf", "cd") for o in ("sum", "prod")])
def test_tree_scalar_path_pair_and_complex_every_program(gu, dtype, op):
    """The scalar tree kernel (operands not 16-B congruent: leaves shifted by the element's
    alignment against the output) on the pair and complex types, EVERY program of 4, 5 and 8 leaves
    with stack depth <= 4 (5 + 13 + 233), swap bits drawn per program: bit-exact vs the oracle.  A
    random 8-leaf depth-4 program once exposed a miscompile of struct-typed stack slots
    (C_FLOAT_COMPLEX, a leaf's words shifted by one); the slots now hold word vectors."""
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    shift = 8 if es == 16 else 4  # the element's own alignment (double / long: 8, float / int: 4)
    n = 5
    pat = po.PAT_TIES if dtype in ("fi", "di") else po.PAT_UNIFORM
    rng = np.random.default_rng(zlib.crc32(f"every-{dtype}-{op}".encode()))
    bad = []
    for nl in (4, 5, 8):
        leaves = [po.fill(n, dtype, pat, 23 + nl, r) for r in range(nl)]
        d = []
        for x in leaves:
            t = gu.empty_dev(n * es + shift)
            t[shift:shift + n * es] = gu.to_dev(x)
            d.append(t)
        out = gu.empty_dev(n * es)
        for comb in all_programs(nl):
            swaps = [int(v) for v in rng.integers(0, 2, nl - 1)]
            rc = ca.reduce_tree(out.data_ptr(), [t.data_ptr() + shift for t in d], comb, swaps, n, DT[dtype], OP[op],
                                gu.stream())
            assert rc == 0
            gu.sync()
            got = gu.from_dev(out, npdt, n)
            ref = tree_ref(leaves, comb, swaps, dtype, op)
            if not np.array_equal(_bits(got), _bits(ref)):
                bad.append((nl, comb, swaps))
    assert not bad, f"{len(bad)} programs differ, e.g. {bad[:3]}"
