"""MPICH baseline allreduces on CPU: oracle and compiled plans vs the
reference's own code.

tests/golden/mpich_manifest.json holds outputs of the reference's
testing/mpich_implementations/all_reduce/{allreduce_ring, allreduce_recursive_doubling,
allreduce_reduce_scatter_allgather, allreduce_recexch}.cpp compiled unchanged against
MPICH 3.3.2 (gen_golden.py mpich).  Bit-exact for every dtype and op.
"""
import hashlib

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po

MODE = {"ring": ca.MODE_MPICH_RING, "rd": ca.MODE_MPICH_RD, "rsag": ca.MODE_MPICH_RSAG,
        "rx": ca.MODE_MPICH_RECEXCH, "krsag": ca.MODE_MPICH_KRSAG, "rm": ca.MODE_MPICH_RMULT}


def _sends(c):
    return [po.fill(c["count"], c["dtype"], c["pattern"], c["seed"], r) for r in range(c["n"])]


def _digest(outs):
    return hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()


def test_manifest_covers_main_cpp_baselines(golden_mpich):
    cases, _ = golden_mpich
    assert len(cases) > 1000
    have = {(c["mode"], c["dtype"], c["op"], c["pattern"]) for c in cases}
    for m in MODE:
        assert (m, "f64", "sum", po.PAT_UNIFORM) in have  # testing/main.cpp's datatype
        assert (m, "f32", "max", po.PAT_TIES) in have
    assert {c["n"] for c in cases} >= {1, 2, 3, 5, 8, 12, 16}


def test_oracle_matches_reference(golden_mpich):
    cases, arrays = golden_mpich
    bad = []
    for c in cases:
        outs = po.mpich_allreduce(c["mode"], _sends(c), c["dtype"], c["op"], k=c["k"], inplace=bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
        elif c["stored"]:
            np.testing.assert_array_equal(np.concatenate(outs), arrays[c["id"]])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_compiled_plans_match_reference(golden_mpich):
    """libchiara's plans for the four baselines, interpreted on CPU, give the reference's bytes."""
    cases, _ = golden_mpich
    bad = []
    for c in cases:
        outs = plan_sim.simulate(MODE[c["mode"]], _sends(c), c["k"], c["b"], c["dtype"], c["op"],
                                 inplace=bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_ties_pattern_detects_operand_order(golden_mpich):
    """The PAT_TIES cases really pin MPICH_do_reduce's running-value-first order: replaying
    recexch / recursive multiplying with the default order (running value second) must
    disagree somewhere."""
    cases, _ = golden_mpich
    rx = [c for c in cases if c["mode"] in ("rx", "rm") and c["pattern"] == po.PAT_TIES and c["n"] >= 4]
    assert rx
    flipped = 0
    for c in rx:
        plans = plan_sim.load_plans(MODE[c["mode"]], c["n"], c["k"], c["b"], c["count"])
        for p in plans:
            for st in p["steps"]:
                st["post"] = [("reduce",) + op[1:] if op[0] == "reduce_sw" else op for op in st["post"]]
        outs = plan_sim.execute(plans, _sends(c), c["dtype"], c["op"], bool(c["inplace"]))
        flipped += _digest(outs) != c["sha256"]
    assert flipped > 0


@pytest.mark.parametrize("mode", sorted(MODE))
def test_plan_step_counts(mode):
    """Step structure follows the reference loops (all ranks agree on the step count)."""
    for n in (1, 2, 3, 6, 8, 13):
        k = 3
        plans = plan_sim.load_plans(MODE[mode], n, k, 0, 100)
        steps = {len(p["steps"]) for p in plans}
        assert len(steps) == 1
        pof2 = 1 << (n.bit_length() - 1)
        if mode == "ring":
            assert steps == {n}  # n-1 reduce-scatter steps + one allgatherv
        elif mode == "rd":
            assert steps == {pof2.bit_length() - 1 + 2}
        elif mode == "rsag":
            assert steps == {2 * (pof2.bit_length() - 1) + 2}


def test_plan_errors():
    with pytest.raises(ValueError):
        plan_sim.simulate(MODE["rx"], [np.zeros(4, np.float32)] * 3, 1, 0, "f32", "sum")
