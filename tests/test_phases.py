"""CHiArA's phases as stand-alone collectives, on CPU: the oracle and libchiara's compiled plans vs the
reference's own code.

testing/custom_implementations/work_dir/reduce_scatter/ keeps each phase of the hierarchical
reduce-scatter as its own function with a DEBUG_MODE self-test main: intra_reduce_scatter_radix_batch
(intra_reduce_scatter_radix.cpp:208, phase 1), inter_reduce_linear (inter_linear_reduce.cpp:11, phase 2)
and intra_scatter_radix_batch (intra_scatter_radix_batch.cpp:10, the reduce-scatter's phase 3).
tests/golden/phases_manifest.json holds their outputs, compiled unchanged against MPICH 3.3.2
(gen_golden.py phases): every divisor b of n = 1 .. 18, k = 2 .. 7, stages with and without a leftover
stage, step-1 folds, in place, and the self-tests' own parameters.  Bit-exact."""
import hashlib

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po

MODE = {"irs": ca.MODE_INTRA_REDUCE_SCATTER, "ilr": ca.MODE_INTER_REDUCE_LINEAR, "isc": ca.MODE_INTRA_SCATTER}


def _sends(c):
    in_n, _ = po.phase_sizes(c["mode"], c["n"], c["b"], c["count"])
    return [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(c["n"])]


def _digest(outs):
    return hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()


def simulate(mode, sends, k, b, dtype, op, rc, inplace=False):
    """Every rank's recv buffer (phase_sizes' output size, zero where the plan writes nothing)."""
    n = len(sends)
    plans = plan_sim.load_plans(MODE[mode], n, k if mode != "ilr" else 2, b, rc)
    if plans[0]["header"]["error"]:
        raise ValueError(f"plan error {plans[0]['header']['error']}")
    _, out_n = po.phase_sizes(mode, n, b, rc)
    if inplace:
        outs = plan_sim.execute(plans, [s.copy() for s in sends], dtype, op, inplace=True)
    else:
        outs = plan_sim.execute(plans, sends, dtype, op,
                                recv_init=[np.zeros(out_n, dtype=sends[0].dtype) for _ in sends])
    return [o[:out_n] for o in outs]


def test_manifest_covers_the_three_phases(golden_phases):
    cases, _ = golden_phases
    assert {c["mode"] for c in cases} == set(MODE)
    geo = {(c["n"], c["b"]) for c in cases}
    nnodes = lambda n, b: n // b  # noqa: E731
    assert any(nnodes(n, b) // b >= 2 for n, b in geo)                        # several stages
    assert any(nnodes(n, b) % b and nnodes(n, b) // b for n, b in geo)        # stages plus a leftover stage
    assert any(nnodes(n, b) < b for n, b in geo)                              # only a leftover stage
    assert any(c["mode"] == "irs" and c["b"] in (3, 5, 6, 9, 12) for c in cases)  # step-1 folds
    assert any(c["mode"] == "irs" and c["inplace"] for c in cases)
    # the self-tests' own parameters
    assert any(c["mode"] == "irs" and (c["k"], c["b"], c["count"]) == (2, 4, 1) for c in cases)
    assert any(c["mode"] == "ilr" and (c["b"], c["count"]) == (2, 1) for c in cases)
    assert any(c["mode"] == "isc" and (c["k"], c["b"], c["count"]) == (7, 9, 7) for c in cases)


def test_oracle_matches_reference(golden_phases):
    cases, arrays = golden_phases
    bad = []
    for c in cases:
        outs = po.phase_collective(c["mode"], _sends(c), c["dtype"], c["op"], c["k"] or 2, c["b"], c["count"],
                                   inplace=bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
        elif c["stored"]:  # raw bytes (pair and complex elements are stored as bytes)
            assert np.concatenate(outs).tobytes() == arrays[c["id"]].tobytes(), c["id"]
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_compiled_plans_match_reference(golden_phases):
    """libchiara's plans for the three phases, interpreted on CPU, give the reference's bytes."""
    cases, _ = golden_phases
    bad = []
    for c in cases:
        outs = simulate(c["mode"], _sends(c), c["k"], c["b"], c["dtype"], c["op"], c["count"], bool(c["inplace"]))
        if _digest(outs) != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:5]}"


def test_intra_scatter_self_test():
    """intra_scatter_radix_batch.cpp's own check (:150-157, :226-233): the node root holds
    100000 * node + 1000 * s + j in block s, every rank of the node must end with block `lane`."""
    n, k, b, rc = 18, 7, 9, 7
    sends = []
    for r in range(n):
        node = r // b
        sends.append(np.array([100000 * node + 1000 * s + j for s in range(b) for j in range(rc)], dtype=np.int32))
    outs = simulate("isc", sends, k, b, "i32", "sum", rc)
    for r in range(n):
        np.testing.assert_array_equal(outs[r], 100000 * (r // b) + 1000 * (r % b) + np.arange(rc, dtype=np.int32))


def test_inter_linear_self_test_pattern():
    """inter_linear_reduce.cpp's self-test input (:136-141: 10000 * rank + 100 * i + j): the root of
    iteration i (node i * b + lane) holds the sum over the lane's ranks; nobody else is written."""
    for n, b in ((8, 2), (12, 2), (18, 3), (16, 4)):
        rc = 3
        nnodes = n // b
        niters = nnodes // b + (1 if nnodes % b else 0)
        irc = rc * b
        sends = [np.array([10000 * r + 100 * i + j for i in range(niters) for j in range(irc)], dtype=np.int32)
                 for r in range(n)]
        outs = simulate("ilr", sends, 0, b, "i32", "sum", rc)
        for r in range(n):
            node, lane = divmod(r, b)
            i, rem = divmod(node - lane, b) if node >= lane else (-1, 1)
            if rem == 0 and 0 <= i < niters:
                want = sum(10000 * (j * b + lane) for j in range(nnodes)) + nnodes * (100 * i + np.arange(irc))
                np.testing.assert_array_equal(outs[r], want.astype(np.int32))
            else:
                assert not outs[r].any()


@pytest.mark.parametrize("n,b", [(6, 2), (12, 3), (16, 4), (8, 1)])
def test_intra_reduce_scatter_equals_group_sums(n, b):
    """Integer SUM: recv[s * IRC] of lane l is chunk s * b + l summed over the group (the self-test's
    pattern rank + 1 + 100 * (i / IRC), intra_reduce_scatter_radix.cpp:584-588)."""
    rc, k = 2, 2
    irc, nnodes = rc * b, n // b
    nstages, nu = nnodes // b, nnodes % b
    sends = [np.array([r + 1 + 100 * (i // irc) for i in range(rc * n)], dtype=np.int32) for r in range(n)]
    outs = simulate("irs", sends, k, b, "i32", "sum", rc)
    for r in range(n):
        node, lane = divmod(r, b)
        group = [node * b + q for q in range(b)]
        for s in range(nstages + (1 if lane < nu else 0)):
            c = s * b + lane
            want = sum(sends[q][c * irc:(c + 1) * irc] for q in group)
            np.testing.assert_array_equal(outs[r][s * irc:(s + 1) * irc], want)


def test_plans_reject_bad_geometry():
    for mode in MODE.values():
        assert ca.parse_plan(ca.describe_plan(mode, 6, 0, 2, 4, 8))["header"]["error"] == 3  # 6 % 4
        assert ca.parse_plan(ca.describe_plan(mode, 4, 0, 2, 0, 8))["header"]["error"] == 1  # b = 0
    assert ca.parse_plan(ca.describe_plan(ca.MODE_INTRA_SCATTER, 4, 0, 1, 2, 8))["header"]["error"] == 1  # k < 2


def test_reference_selftest_outputs_agree_with_the_oracle():
    """tests/golden/selftest_outputs.json (the reference's DEBUG_MODE mains, run here; the GPU test runs
    the same mains on libchiara) checked on CPU: the scatter's RESULT: PASS, and every AFTER buffer the
    mains print equals the oracle on the mains' own inputs."""
    import json
    import os
    import re

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "selftest_outputs.json")) as f:
        runs = json.load(f)["runs"]
    ints = lambda s: [int(x) for x in re.findall(r"-?\d+", s)]  # noqa: E731
    for key, run in runs.items():
        n, lines = run["nranks"], run["lines"]
        if run["binary"] not in ("intra_reduce_scatter_radix", "inter_linear_reduce", "intra_scatter_radix_batch"):
            continue  # the other mains: tests/test_selftests.py
        if run["binary"] == "intra_scatter_radix_batch":
            assert lines["0"][-1].startswith("RESULT: PASS"), key
        elif run["binary"] == "inter_linear_reduce":
            b, rc = (int(a) for a in run["args"])
            in_n, out_n = po.phase_sizes("ilr", n, b, rc)
            irc = rc * b
            sends = [np.array([10000 * r + 100 * (i // irc) + i % irc for i in range(in_n)], dtype=np.int32)
                     for r in range(n)]
            want = po.phase_collective("ilr", sends, "i32", "sum", 2, b, rc)
            for r in range(n):
                after = lines[str(r)][lines[str(r)].index(f"== AFTER  rank {r} (rc=0) ==") + 2:]
                got = [v for ln in after for v in ints(ln.split(":", 1)[1])][:irc]
                root = any(i * b + r % b == r // b for i in range(in_n // irc))
                assert got == (want[r].tolist() if root else [-777777] * irc), (key, r)
        else:
            rc, k, b = (int(a) for a in run["args"])
            in_n, out_n = po.phase_sizes("irs", n, b, rc)
            sends = [np.array([r + 1 + 100 * (i // (rc * b)) for i in range(in_n)], dtype=np.int32) for r in range(n)]
            want = po.phase_collective("irs", sends, "i32", "sum", k, b, rc)
            for r in range(n):
                assert ints(lines[str(r)][-1]) == want[r].tolist(), (key, r)


def test_buffers_each_rank_touches():
    """What each rank's plan reads and writes (chr_plan_describe header): the scatter reads `send` on node
    roots only and the linear reduce writes `recv` on iteration roots only -- the other ranks may pass NULL,
    as the reference's own callers do (intra_scatter_radix_batch.cpp:213) or could (inter_linear_reduce.cpp
    never touches recvbuf off the roots).  Phase 1 writes the leftover stage's chunk on lanes < nu only."""
    n, b, rc = 12, 2, 5  # nnodes 6, nstages 3, nu 0; niters 3
    for r in range(n):
        h = ca.parse_plan(ca.describe_plan(ca.MODE_INTRA_SCATTER, n, r, 2, b, rc))["header"]
        node, lane = divmod(r, b)
        assert (h["send"], h["recv"]) == ((b * rc if lane == node % b else 0), rc)
        h = ca.parse_plan(ca.describe_plan(ca.MODE_INTER_REDUCE_LINEAR, n, r, 2, b, rc))["header"]
        root = any(i * b + lane == node for i in range(3))
        assert (h["send"], h["recv"]) == (3 * rc * b, rc * b if root else 0)
    n, b = 12, 4  # nnodes 3 < b: only a leftover stage, nu = 3
    for r in range(n):
        h = ca.parse_plan(ca.describe_plan(ca.MODE_INTRA_REDUCE_SCATTER, n, r, 2, b, rc))["header"]
        assert (h["send"], h["recv"]) == (rc * n, rc * b if r % b < 3 else 0)
