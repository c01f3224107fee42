"""The MPICH baselines with a user-defined op, on CPU: oracle and compiled plans vs the reference itself.

tests/golden/usermpich_outputs.npz holds the outputs of the reference's testing/mpich_implementations/{all_reduce,
reduce_scatter}/*.cpp compiled unchanged against MPICH 3.3.2 with MPI_Op_create(halfadd) -- inout = in * 0.5f + inout
on MPI_FLOAT, non-commutative arithmetic -- created non-commutative (user_halfadd) and commutative (user_halfadd_c),
with every rank's return code (gen_golden.py usermpich).  The baselines branch on MPI_Op_commutative: recursive
doubling keeps rank order for a non-commutative op (allreduce_recursive_doubling.cpp:69-80,
reduce_scatter_recursive_doubling.cpp:134-160), k-reduce-scatter-allgather and recursive multiplying at a size that is
not a power of k refuse it with MPI_ERR_OP (allreduce_k_reduce_scatter_allgather.cpp:278-283,
allreduce_recursive_multiplying.cpp:43-49).  Both the oracle and libchiara's plans must reproduce every output bit
for bit and every refusal."""
import json
import os

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "usermpich_manifest.json")))
FIX = np.load(os.path.join(HERE, "golden", "usermpich_outputs.npz"), allow_pickle=False)
MPI_ERR_OP = 9  # MPICH 3.3.2's class code, as the reference returned it (ref_rc)

MODE = {"ring": ca.MODE_MPICH_RING, "rd": ca.MODE_MPICH_RD, "rsag": ca.MODE_MPICH_RSAG,
        "rx": ca.MODE_MPICH_RECEXCH, "krsag": ca.MODE_MPICH_KRSAG, "rm": ca.MODE_MPICH_RMULT,
        "rs_radix": ca.MODE_MPICH_RS_RADIX, "rs_halving": ca.MODE_MPICH_RS_HALVING,
        "rs_doubling": ca.MODE_MPICH_RS_DOUBLING, "rs_pairwise": ca.MODE_MPICH_RS_PAIRWISE}


def refused(c):
    return MPI_ERR_OP in c["ref_rc"]


def sends_of(c):
    n = c["n"]
    in_n = c["count"] * n if c["mode"].startswith("rs_") else c["count"]
    return [po.fill(in_n, "f32", c["pattern"], c["seed"], r) for r in range(n)]


def oracle_outputs(c):
    sends, ip = sends_of(c), bool(c["inplace"])
    if c["mode"].startswith("rs_"):
        return po.mpich_reduce_scatter(c["mode"], sends, "f32", c["op"], k=c["k"], inplace=ip)
    return po.mpich_allreduce(c["mode"], sends, "f32", c["op"], k=c["k"], inplace=ip)


def test_fixture_covers_both_branches():
    """Both creations, every baseline, refusals where the reference gives them, and the commutative flag visible
    in the bits (the same function, created two ways, gives different recursive-doubling outputs)."""
    cases = MAN["cases"]
    assert {c["mode"] for c in cases} == set(MODE) and {c["op"] for c in cases} == {"user_halfadd", "user_halfadd_c"}
    ref = {(c["mode"], c["op"]) for c in cases if refused(c)}
    assert ref == {("krsag", "user_halfadd"), ("rm", "user_halfadd")}
    key = lambda c: (c["mode"], c["n"], c["k"], c["b"], c["count"])  # noqa: E731  (in place or not: same bits)
    comm = {key(c): c for c in cases if c["op"] == "user_halfadd_c"}
    differ = 0
    for c in cases:
        if c["op"] == "user_halfadd" and c["mode"] in ("rd", "rs_doubling") and c["n"] >= 3:
            twin = comm[key(c)]
            differ += not np.array_equal(FIX[c["id"]].view(np.uint32), FIX[twin["id"]].view(np.uint32))
    assert differ > 0


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["id"])
def test_oracle_matches_reference(case):
    if refused(case):
        with pytest.raises(ValueError) as e:
            oracle_outputs(case)
        assert e.value.args[1] == po.ORC_ERR_OP
        return
    got = np.concatenate([np.asarray(o).ravel() for o in oracle_outputs(case)])
    assert np.array_equal(got.view(np.uint32), FIX[case["id"]].view(np.uint32))


def test_compiled_plans_match_reference():
    """libchiara's plans for every case (chr_plan_describe_op with the op's commutativity), interpreted on CPU with
    the oracle's MPI_Reduce_local: the reference's bytes, and CHR_ERR_UNSUPPORTED where it returns MPI_ERR_OP."""
    bad = []
    for c in MAN["cases"]:
        try:
            outs = plan_sim.simulate(MODE[c["mode"]], sends_of(c), c["k"], c["b"], "f32", c["op"],
                                     inplace=bool(c["inplace"]))
        except ValueError as e:
            if not (refused(c) and e.args[1] == ca.ERR_UNSUPPORTED):
                bad.append((c["id"], str(e)))
            continue
        if refused(c) or not np.array_equal(np.concatenate(outs).view(np.uint32), FIX[c["id"]].view(np.uint32)):
            bad.append(c["id"])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_non_commutative_plans_differ_only_where_the_reference_branches():
    """Plan text of a non-commutative op equals the commutative one except for recursive doubling's swapped combines
    and the refusals."""
    for mode, n, k in (("ring", 5, 0), ("rsag", 6, 0), ("rx", 7, 3), ("rs_halving", 6, 0), ("rs_pairwise", 5, 0),
                       ("rs_radix", 9, 3), ("rm", 9, 3)):
        for r in range(n):
            a = ca.describe_plan(MODE[mode], n, r, k, 0, 64, 1, None, True)
            assert a == ca.describe_plan(MODE[mode], n, r, k, 0, 64, 1, None, False), (mode, n, r)
    swapped = [ca.describe_plan(MODE["rd"], 8, r, 0, 0, 64, 1, None, False).count("reduce_sw") for r in range(8)]
    assert swapped == [3, 2, 2, 1, 2, 1, 1, 0]  # the partners above each rank at distances 1, 2, 4
    for mode, n, k in (("krsag", 4, 2), ("rm", 6, 2)):
        assert ca.parse_plan(ca.describe_plan(MODE[mode], n, 0, k, 0, 64, 1, None, False))["header"]["error"] == \
            ca.ERR_UNSUPPORTED
