"""User-defined reduction ops on the device (chr_op_create, ABI 11) vs the reference and the oracle.

The reference is generic over MPI_Op (all_reduce_radix_batch.cpp:202-204), user-defined ops included: here the op is
MPI_Op_create(halfadd, commute = 0) -- inout = in * 0.5f + inout on float, non-commutative, so every operand order
shows in the bits -- as the caller's own device code (tests/userop/halfadd_op.hip through include/chiara_user_op.hpp).
The collectives must reproduce the reference's outputs for the same op bit for bit (tests/golden/userop_outputs.npz:
the reference compiled unchanged against MPICH with that MPI_Op), and every fold / tree the library evaluates must
match the oracle's restatement (chiara_oracle.c ORC_USER_HALFADD).  The MPICH baselines take user ops as the
reference's do: branching on MPI_Op_commutative, so the same function registered commutative and non-commutative
(tests/golden/usermpich_outputs.npz, the reference run with both) gives different bits, and refusing a
non-commutative op where the reference returns MPI_ERR_OP (CHR_ERR_UNSUPPORTED, as for a launcher that refuses the
call)."""
import ctypes
import json
import os

import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po
from tree_util import random_program, tree_ref

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
USEROP_SO = os.path.join(HERE, "userop", "libhalfadd_op.so")
MAN = json.load(open(os.path.join(HERE, "golden", "userop_manifest.json")))
FIX = np.load(os.path.join(HERE, "golden", "userop_outputs.npz"), allow_pickle=False)
MMAN = json.load(open(os.path.join(HERE, "golden", "usermpich_manifest.json")))
MFIX = np.load(os.path.join(HERE, "golden", "usermpich_outputs.npz"), allow_pickle=False)
OPN = "user_halfadd"


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


@pytest.fixture(scope="module")
def ops():
    """(halfadd, refusing, halfadd registered commutative) op codes, registered from the test's own code object and
    freed at the end."""
    assert os.path.exists(USEROP_SO), f"{USEROP_SO} missing: make -C tests/userop (__graft_entry__.build())"
    lib = ctypes.CDLL(USEROP_SO)
    half = ca.op_create(ctypes.cast(lib.chr_test_halfadd, ctypes.c_void_p).value)
    refuse = ca.op_create(ctypes.cast(lib.chr_test_refuse, ctypes.c_void_p).value)
    half_c = ca.op_create(ctypes.cast(lib.chr_test_halfadd, ctypes.c_void_p).value, commute=True)
    yield half, refuse, half_c
    assert ca.op_free(half) == 0 and ca.op_free(refuse) == 0 and ca.op_free(half_c) == 0


@pytest.fixture(scope="module")
def groups():
    cache = {}

    def get(n):
        if n not in cache:
            cache[n] = ca.LocalGroup(n, 0)
        return cache[n]

    yield get
    for g in cache.values():
        g.destroy()


def _u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


# ---- the folds and trees every collective is built from ---------------------------------------

def _chain_ref(acc, ins, running_first):
    """MPI_Reduce_local chained over ins: acc = in_j o acc, or with running_first acc = acc o in_j (MPICH_do_reduce
    order, the library's REDUCE_RUNNING_FIRST flag)."""
    v = acc.copy()
    for x in ins:
        if running_first:
            y = x.copy()
            po.reduce_local(v, y, "f32", OPN)
            v = y
        else:
            po.reduce_local(x, v, "f32", OPN)
    return v


@pytest.mark.parametrize("m", [0, 1, 3, 8, 17])
@pytest.mark.parametrize("n", [1, 1000, 300001])
def test_fold_matches_oracle(gu, ops, m, n):
    """chr_reduce_multi_ex with a user op: m incoming buckets into the accumulator, both operand orders, fan-in above
    the functor kernel's kMaxIns (17: two launches), out of place and in place (out = acc)."""
    half = ops[0]
    acc = po.fill(n, "f32", po.PAT_UNIFORM, 21, 0)
    ins = [po.fill(n, "f32", po.PAT_UNIFORM, 21, j + 1) for j in range(m)]
    d_ins = [gu.to_dev(x) for x in ins]
    for flags in (0, ca.REDUCE_RUNNING_FIRST):
        want = _chain_ref(acc, ins, bool(flags))
        if m > 0:
            assert po.reduce_multi(acc.copy(), ins, "f32", OPN).tobytes() == _chain_ref(acc, ins, False).tobytes()
        for inplace in (False, True):
            d_acc = gu.to_dev(acc)
            d_out = d_acc if inplace else gu.empty_dev(acc.nbytes)
            assert ca.reduce_multi_ex(d_out, d_acc, d_ins, n, ca.FLOAT32, half, flags, gu.stream()) == 0
            gu.sync()
            np.testing.assert_array_equal(_u32(gu.from_dev(d_out, np.float32, n)), _u32(want))


def test_reduce_local_matches_oracle(gu, ops):
    half = ops[0]
    n = 77777
    x = po.fill(n, "f32", po.PAT_UNIFORM, 5, 0)
    y = po.fill(n, "f32", po.PAT_UNIFORM, 5, 1)
    dx, dy = gu.to_dev(x), gu.to_dev(y)
    assert ca.reduce_local(dx, dy, n, ca.FLOAT32, half, gu.stream()) == 0
    gu.sync()
    np.testing.assert_array_equal(_u32(gu.from_dev(dy, np.float32, n)), _u32(po.reduce_local(x, y.copy(), "f32", OPN)))


C4_TREE = ([0, 1, 1, 1, 0, 1, 1, 2], [0] * 7)                     # the flat schedule's k=4, b=4 tree
SWAP_TREE = ([0, 1, 1, 1, 0, 1, 1, 2], [1, 0, 1, 0, 1, 0, 1])     # running-value-first combines


def test_trees_match_oracle(gu, ops):
    """chr_reduce_tree with a user op: the post-order program evaluated fold by fold (user_ops.cpp user_tree), fixed
    and random programs of 1..8 leaves with random swap bits, out of place and into a leaf."""
    half = ops[0]
    rng = np.random.default_rng(7)
    progs = [C4_TREE, SWAP_TREE, ([0], [])] + [random_program(rng, nl) for nl in (2, 3, 5, 6, 7, 8, 8)]
    n = 65537
    for comb, swaps in progs:
        leaves = [po.fill(n, "f32", po.PAT_UNIFORM, 13, r) for r in range(len(comb))]
        want = tree_ref(leaves, comb, swaps, "f32", OPN)
        for into_leaf in (None, 0):
            d = [gu.to_dev(x) for x in leaves]
            out = gu.empty_dev(n * 4) if into_leaf is None else d[into_leaf]
            assert ca.reduce_tree(out, d, comb, swaps, n, ca.FLOAT32, half, gu.stream()) == 0
            gu.sync()
            np.testing.assert_array_equal(_u32(gu.from_dev(out, np.float32, n)), _u32(want), err_msg=str(comb))


def test_tree_batch_matches_oracle(gu, ops):
    half = ops[0]
    rng = np.random.default_rng(9)
    n, nt, nl = 4099, 5, 6
    progs = [random_program(rng, nl) for _ in range(nt)]
    leaves = [[po.fill(n, "f32", po.PAT_UNIFORM, 40 + t, r) for r in range(nl)] for t in range(nt)]
    d_leaves = [[gu.to_dev(x) for x in lv] for lv in leaves]
    outs = [gu.empty_dev(n * 4) for _ in range(nt)]
    assert ca.reduce_tree_batch(outs, d_leaves, [c for c, _ in progs], [s for _, s in progs], n, ca.FLOAT32, half,
                                gu.stream()) == 0
    gu.sync()
    for t, (comb, swaps) in enumerate(progs):
        np.testing.assert_array_equal(_u32(gu.from_dev(outs[t], np.float32, n)),
                                      _u32(tree_ref(leaves[t], comb, swaps, "f32", OPN)))


# ---- the collectives vs the reference ----------------------------------------------------------

PHASE_MODE = {"irs": ca.MODE_INTRA_REDUCE_SCATTER, "ilr": ca.MODE_INTER_REDUCE_LINEAR}


UDT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32}  # the types the test op's launcher implements


def _run_case(gu, g, c, op):
    """Every rank's output of golden case c through the local group (rank-major, as the fixture stores them)."""
    n, k, b, count, mode, ip = c["n"], c["k"], c["b"], c["count"], c["mode"], bool(c["inplace"])
    dt, npdt = c["dtype"], po.NP_DTYPES[c["dtype"]]
    es = np.dtype(npdt).itemsize
    if mode in PHASE_MODE:
        in_n, out_n = po.phase_sizes(mode, n, b, count)
    else:
        in_n, out_n = (count * n if mode == "rs" else count), count
    sends = [po.fill(in_n, dt, c["pattern"], c["seed"], r, in_n) for r in range(n)]
    if ip:
        d_recv, d_send = [gu.to_dev(s) for s in sends], [ca.IN_PLACE] * n
    else:
        d_recv, d_send = [gu.empty_dev(out_n * es) for _ in range(n)], [gu.to_dev(s) for s in sends]
    if mode in PHASE_MODE:
        rc = g.phase_collective(PHASE_MODE[mode], d_send, d_recv, count, UDT[dt], op, k, b)
    else:
        fn = g.all_reduce_radix_batch if mode == "ar" else g.reduce_scatter_radix_batch
        rc = fn(d_send, d_recv, count, UDT[dt], op, k, b)
    assert rc == 0, (c["id"], rc)
    return np.concatenate([gu.from_dev(d, npdt, out_n) for d in d_recv])


@pytest.mark.parametrize("schedule", ["flat", "exact"])
def test_collectives_match_reference_golden(gu, ops, groups, schedule):
    """Every user-op golden case of the reference (radix/batch allreduce and reduce-scatter at every batch size b
    that divides n, k = 2..4, in place and not; CHiArA's phases; float, double and int32 through one launcher that
    switches on the type) bit-exact on the device.  The flat schedule evaluates
    each chunk as one expression tree, the exact one replays the reference's messages -- both must land on the
    reference's operand order."""
    half = ops[0]
    bad = []
    for c in MAN["cases"]:
        g = groups(c["n"])
        g.set_schedule(ca.SCHEDULE_EXACT if schedule == "exact" else ca.SCHEDULE_FLAT)
        try:
            got = _run_case(gu, g, c, half)
        finally:
            g.set_schedule(ca.SCHEDULE_FLAT)
        if got.dtype != FIX[c["id"]].dtype or not np.array_equal(got.view(np.uint8), FIX[c["id"]].view(np.uint8)):
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("n,k,b,slices", [(8, 4, 4, 1), (8, 2, 8, 4), (6, 3, 2, 2)])
def test_collectives_large_vs_oracle(gu, ops, groups, n, k, b, slices):
    """MiB-sized buckets (the scratch-backed tree evaluation at size, sliced plans): bit-exact vs the oracle."""
    half = ops[0]
    count = n * ((1 << 17) + 5)
    sends = [po.fill(count, "f32", po.PAT_UNIFORM, 17, r) for r in range(n)]
    g = groups(n)
    g.set_slices(slices)
    try:
        d_send = [gu.to_dev(s) for s in sends]
        d_recv = [gu.empty_dev(count * 4) for _ in range(n)]
        assert g.all_reduce_radix_batch(d_send, d_recv, count, ca.FLOAT32, half, k, b) == 0
        want = po.allreduce_radix_batch(sends, k, b, "f32", OPN)
        for r in range(n):
            np.testing.assert_array_equal(_u32(gu.from_dev(d_recv[r], np.float32, count)), _u32(want[r]))
    finally:
        g.set_slices(1)


def test_comm_single_rank_with_graphs(gu, ops):
    """The RCCL communicator path with a user op at nranks = 1, graphs on (user-op calls run eagerly: the launcher
    is the caller's and may not be capturable) -- then a predefined op still replays its graph."""
    import torch

    half = ops[0]
    comm = ca.Comm(1, ca.get_unique_id(), 0, 0)
    try:
        comm.set_graphs(True)
        x = po.fill(4096, "f32", po.PAT_UNIFORM, 3, 0)
        ds, dr = gu.to_dev(x), gu.empty_dev(x.nbytes)
        for op in (half, half, ca.SUM, ca.SUM):
            assert ca.all_reduce_radix_batch(ds, dr, x.size, ca.FLOAT32, op, comm, 2, 1) == 0
            torch.cuda.synchronize()
            np.testing.assert_array_equal(_u32(gu.from_dev(dr, np.float32, x.size)), _u32(x))
    finally:
        comm.set_graphs(False)
        comm.destroy()


MPICH_AR = {"ring": ca.MODE_MPICH_RING, "rd": ca.MODE_MPICH_RD, "rsag": ca.MODE_MPICH_RSAG,
            "rx": ca.MODE_MPICH_RECEXCH, "krsag": ca.MODE_MPICH_KRSAG, "rm": ca.MODE_MPICH_RMULT}
MPICH_RS = {"rs_radix": ca.MODE_MPICH_RS_RADIX, "rs_halving": ca.MODE_MPICH_RS_HALVING,
            "rs_doubling": ca.MODE_MPICH_RS_DOUBLING, "rs_pairwise": ca.MODE_MPICH_RS_PAIRWISE}


def test_mpich_baselines_match_reference_golden(gu, ops, groups):
    """The ten MPICH baselines with the user op registered non-commutative and commutative: every golden case of the
    reference (gen_golden.py usermpich) bit-exact on the device, and CHR_ERR_UNSUPPORTED wherever the reference
    returned MPI_ERR_OP."""
    half, _, half_c = ops
    bad = []
    for c in MMAN["cases"]:
        n, count, ip = c["n"], c["count"], bool(c["inplace"])
        op = half if c["op"] == "user_halfadd" else half_c
        rs = c["mode"] in MPICH_RS
        in_n = count * n if rs else count
        sends = [po.fill(in_n, "f32", c["pattern"], c["seed"], r) for r in range(n)]
        if ip:
            d_recv, d_send = [gu.to_dev(s) for s in sends], [ca.IN_PLACE] * n
        else:
            d_recv, d_send = [gu.empty_dev(count * 4) for _ in range(n)], [gu.to_dev(s) for s in sends]
        g = groups(n)
        if rs:
            rc = g.reduce_scatter_mpich(MPICH_RS[c["mode"]], d_send, d_recv, count, ca.FLOAT32, op, c["k"])
        else:
            rc = g.allreduce_mpich(MPICH_AR[c["mode"]], d_send, d_recv, count, ca.FLOAT32, op, c["k"], c["b"])
        if 9 in c["ref_rc"]:  # the reference's MPI_ERR_OP
            if rc != ca.ERR_UNSUPPORTED:
                bad.append((c["id"], rc))
            continue
        got = np.concatenate([gu.from_dev(d, np.float32, count) for d in d_recv])
        if rc != 0 or not np.array_equal(_u32(got), _u32(MFIX[c["id"]])):
            bad.append((c["id"], rc))
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


# ---- refusals ---------------------------------------------------------------------------------

def test_refusals(gu, ops, groups):
    """The reference's MPI_ERR_OP for a non-commutative op (k-reduce-scatter-allgather; recursive multiplying at a
    size that is not a power of k) is CHR_ERR_UNSUPPORTED.  A launcher that refuses a call hands its verdict back
    (CHR_ERR_UNSUPPORTED), and a freed or never-created op code is CHR_ERR_INVALID_ARG -- for the kernels and the
    collectives."""
    half, refuse = ops[:2]
    n = 4
    g = groups(n)
    d = [gu.empty_dev(64 * 4) for _ in range(n)]
    dr = [gu.empty_dev(64 * 4) for _ in range(n)]
    assert g.allreduce_mpich(ca.MODE_MPICH_KRSAG, d, dr, 64, ca.FLOAT32, half, 2, 0) == ca.ERR_UNSUPPORTED
    assert groups(6).allreduce_mpich(ca.MODE_MPICH_RMULT, [gu.empty_dev(64 * 4) for _ in range(6)],
                                     [gu.empty_dev(64 * 4) for _ in range(6)], 64, ca.FLOAT32, half, 4, 0) == \
        ca.ERR_UNSUPPORTED  # 6 is not a power of 4
    assert g.all_reduce_radix_batch(d, dr, 64, ca.FLOAT32, refuse, 2, 2) == ca.ERR_UNSUPPORTED
    assert ca.reduce_local(d[0], d[1], 64, ca.FLOAT32, refuse, gu.stream()) == ca.ERR_UNSUPPORTED
    # a type the op's launcher does not implement: its verdict, for the kernels and the collectives
    assert ca.reduce_local(d[0], d[1], 64, ca.INT64, half, gu.stream()) == ca.ERR_UNSUPPORTED
    assert g.all_reduce_radix_batch(d, dr, 32, ca.INT64, half, 2, 2) == ca.ERR_UNSUPPORTED
    gu.sync()
    lib = ctypes.CDLL(USEROP_SO)
    tmp = ca.op_create(ctypes.cast(lib.chr_test_halfadd, ctypes.c_void_p).value)
    assert tmp not in (half, refuse) and ca.op_free(tmp) == 0
    assert ca.op_free(tmp) == ca.ERR_INVALID_ARG
    assert ca.reduce_local(d[0], d[1], 64, ca.FLOAT32, tmp, gu.stream()) == ca.ERR_INVALID_ARG
    assert g.all_reduce_radix_batch(d, dr, 64, ca.FLOAT32, tmp, 2, 2) == ca.ERR_INVALID_ARG
    assert ca.reduce_local(d[0], d[1], 64, ca.FLOAT32, 127, gu.stream()) == ca.ERR_INVALID_ARG
    # a launcher defined for one type (CHR_DEFINE_USER_OP_FOR): that type runs, any other is refused
    isum = ca.op_create(ctypes.cast(lib.chr_test_isum, ctypes.c_void_p).value, commute=True)
    try:
        x = np.arange(-500, 500, dtype=np.int32)
        y = (np.arange(1000, dtype=np.int32) * 7919).astype(np.int32)
        dx, dy = gu.to_dev(x), gu.to_dev(y)
        assert ca.reduce_local(dx, dy, 1000, ca.INT32, isum, gu.stream()) == 0
        assert ca.reduce_local(dx, dy, 250, ca.FLOAT32, isum, gu.stream()) == ca.ERR_UNSUPPORTED
        gu.sync()
        np.testing.assert_array_equal(gu.from_dev(dy, np.int32, 1000), x + y)
    finally:
        ca.op_free(isum)
    # the registry hands the freed code out again, still live for the next call
    again = ca.op_create(ctypes.cast(lib.chr_test_halfadd, ctypes.c_void_p).value)
    try:
        assert ca.reduce_local(d[0], d[1], 64, ca.FLOAT32, again, gu.stream()) == 0
        gu.sync()
    finally:
        ca.op_free(again)
