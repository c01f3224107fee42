"""MPICH baseline reduce-scatters on CPU: the oracle and libchiara's compiled plans vs the
reference's own code.

tests/golden/rsmpich_manifest.json holds outputs of the reference's
testing/mpich_implementations/reduce_scatter/{reduce_scatter_radix, reduce_scatter_recursive_halving,
reduce_scatter_recursive_doubling, reduce_scatter_pairwise}.cpp compiled unchanged against MPICH 3.3.2
(gen_golden.py rsmpich): the baselines that directory's main.cpp times.  Bit-exact for every dtype and
op, in place and not, n = 1..16 (recursive doubling's relays for non-powers of two included)."""
import hashlib

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po

MODE = {"rs_radix": ca.MODE_MPICH_RS_RADIX, "rs_halving": ca.MODE_MPICH_RS_HALVING,
        "rs_doubling": ca.MODE_MPICH_RS_DOUBLING, "rs_pairwise": ca.MODE_MPICH_RS_PAIRWISE}


def _sends(c):
    return [po.fill(c["count"] * c["n"], c["dtype"], c["pattern"], c["seed"], r) for r in range(c["n"])]


def _digest(outs):
    return hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()


def test_manifest_covers_the_four_baselines(golden_rsmpich):
    cases, _ = golden_rsmpich
    assert {c["mode"] for c in cases} == set(MODE)
    assert {c["n"] for c in cases} >= {1, 2, 3, 5, 6, 7, 8, 9, 12, 16}
    for m in MODE:
        assert any(c["mode"] == m and c["dtype"] == "f64" and c["op"] == "sum" for c in cases)  # main.cpp's
        assert any(c["mode"] == m and c["inplace"] for c in cases)
    ints = [c for c in cases if c["dtype"] in ("i32", "i64", "u16")]
    assert ints and all(c["n_diff_vs_lib"] == 0 for c in ints)  # == MPI_Reduce_scatter_block


def test_oracle_matches_reference(golden_rsmpich):
    cases, arrays = golden_rsmpich
    bad = []
    for c in cases:
        outs = po.mpich_reduce_scatter(c["mode"], _sends(c), c["dtype"], c["op"], k=c["k"] or 2,
                                       inplace=bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
        elif c["stored"]:
            np.testing.assert_array_equal(np.concatenate(outs), arrays[c["id"]])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_compiled_plans_match_reference(golden_rsmpich):
    """libchiara's plans for the four baselines, interpreted on CPU, give the reference's bytes."""
    cases, _ = golden_rsmpich
    bad = []
    for c in cases:
        outs = plan_sim.simulate(MODE[c["mode"]], _sends(c), c["k"], 0, c["dtype"], c["op"],
                                 inplace=bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("n", [3, 5, 6, 7, 12])
def test_recursive_doubling_relays_for_non_powers_of_two(n):
    """reduce_scatter_recursive_doubling.cpp:106-130: ranks without a partner at distance `mask` get
    their blocks relayed down the subtree -- the plans carry those relay steps (aligned on every
    rank), and the result is the exact integer reduce-scatter."""
    plans = plan_sim.load_plans(ca.MODE_MPICH_RS_DOUBLING, n, 0, 0, 5)
    assert any(st["label"] == "rd-relay" and (st["sends"] or st["recvs"]) for p in plans for st in p["steps"])
    sends = [po.fill(5 * n, "i32", po.PAT_UNIFORM, 9, r) for r in range(n)]
    total = (np.stack(sends).astype(np.int64).sum(axis=0) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    outs = plan_sim.simulate(ca.MODE_MPICH_RS_DOUBLING, sends, 0, 0, "i32", "sum")
    for r in range(n):
        np.testing.assert_array_equal(outs[r], total[r * 5:(r + 1) * 5])
