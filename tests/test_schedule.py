"""Schedule compiler (host C++, via chr_plan_describe) on CPU: every golden geometry's
compiled plans, interpreted with numpy, reproduce the oracle / reference bit-exactly."""
import hashlib

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po


def _inputs(c):
    n = c["n"]
    in_n = c["count"] if c["mode"] == "ar" else c["count"] * n
    return [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]


def test_plans_match_reference_golden(golden):
    cases, _ = golden
    bad = []
    for c in cases:
        if c["count"] * c["n"] > (1 << 16):
            continue  # the large hash-only cases are covered on the GPU
        mode = ca.MODE_ALLREDUCE if c["mode"] == "ar" else ca.MODE_REDUCE_SCATTER
        outs = plan_sim.simulate(mode, _inputs(c), c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
        h = hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()
        if h != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} plan/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 2), (8, 4, 8), (8, 3, 4), (2, 2, 1), (2, 2, 2), (16, 4, 4),
                                   (32, 4, 4), (24, 3, 4), (12, 5, 6), (20, 3, 5), (27, 3, 3)])
def test_plans_match_oracle_wider_grid(n, k, b):
    cnt = n * 6
    sends = [po.fill(cnt, "f32", 0, 77, r) for r in range(n)]
    ref = po.allreduce_radix_batch(sends, k, b, "f32", "sum")
    got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, k, b, "f32", "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), ref[r].view(np.uint32))
    sends = [po.fill(cnt, "bf16", 0, 78, r) for r in range(n)]
    ref = po.reduce_scatter_radix_batch(sends, k, b, "bf16", "sum")
    got = plan_sim.simulate(ca.MODE_REDUCE_SCATTER, sends, k, b, "bf16", "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r], ref[r])


def test_plan_errors_match_reference_preconditions():
    h = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 2, 2, 131))["header"]
    assert h["error"] == 2  # count % nranks
    h = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 6, 0, 2, 4, 24))["header"]
    assert h["error"] == 3  # nranks % b
    h = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 1, 2, 16))["header"]
    assert h["error"] == 1  # k < 2


def test_plan_shape_c4():
    """C4 geometry (n=8, k=4, b=4): one recexch phase with k-1=3 concurrent neighbours,
    one fused 3-input reduction per active lane, 1-input lane reduction at the roots."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 20))
    assert p["header"]["k"] == 4 and p["header"]["steps"] == 5
    ph = [s for s in p["steps"] if s["label"].startswith("recexch")]
    assert len(ph) == 1 and len(ph[0]["recvs"]) == 3 and len(ph[0]["sends"]) == 1
    red = [op for op in ph[0]["post"] if op[0] == "reduce"]
    assert len(red) == 1 and len(red[0][4]) == 3
    lane = [s for s in p["steps"] if s["label"] == "inter-lane-reduce"][0]
    assert len(lane["recvs"]) == 1 and lane["post"][0][0] == "reduce"
