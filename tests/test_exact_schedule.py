"""The `exact` schedule (CHR_SCHEDULE_EXACT) on CPU: the reference's communication pattern end
to end -- phases 0-2 plus its inter-node bcast and intra-node k-port Bruck allgather
(all_reduce_radix_batch.cpp:552-756) or its k-nomial scatter (reduce_scatter_radix_batch.cpp
:572-627).

Pinned two ways:
  * bytes per ordered GPU pair equal the REAL reference's, from its PMPI message trace
    (tests/golden/msg_trace.json, tests/golden/gen_trace.py) for every traced geometry;
  * results bit-exact against the golden vectors (plans interpreted by plan_sim)."""
import collections
import hashlib
import json
import os

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))


def _traces():
    with open(os.path.join(HERE, "golden", "msg_trace.json")) as f:
        return json.load(f)["cases"]


def _pair_bytes_trace(c):
    out = collections.Counter()
    for r, msgs in enumerate(c["ranks"]):
        for d, peer, nbytes in msgs:
            if d == 0:
                out[(r, peer)] += nbytes
    return out


def _pair_bytes_plan(mode, n, k, b, count, es):
    out = collections.Counter()
    for r in range(n):
        p = ca.parse_plan(ca.describe_plan(mode, n, r, k, b, count, 1, ca.SCHEDULE_EXACT))
        assert p["header"]["error"] == 0 and p["header"]["schedule"] == ca.SCHEDULE_EXACT
        for st in p["steps"]:
            for peer, _, cnt in st["sends"]:
                out[(r, peer)] += cnt * es
    return out


def test_pair_bytes_match_reference_trace():
    bad = []
    cases = _traces()
    assert len(cases) >= 150
    for c in cases:
        mode = ca.MODE_ALLREDUCE if c["mode"] == "ar" else ca.MODE_REDUCE_SCATTER
        got = _pair_bytes_plan(mode, c["n"], c["k"], c["b"], c["count"], c["elem_bytes"])
        want = _pair_bytes_trace(c)
        if got != want:
            bad.append((c["mode"], c["n"], c["k"], c["b"]))
    assert not bad, f"{len(bad)} geometries differ from the reference's traffic, e.g. {bad[:6]}"


def _tail_messages(mode, n, k, b, count, r):
    p = ca.parse_plan(ca.describe_plan(mode, n, r, k, b, count, 1, ca.SCHEDULE_EXACT))
    tail = [st for st in p["steps"] if any(x in st["label"] for x in ("bcast", "bruck", "kscat"))]
    return sorted([(0, peer, cnt * 4) for st in tail for peer, _, cnt in st["sends"]] +
                  [(1, peer, cnt * 4) for st in tail for peer, _, cnt in st["recvs"]])


def test_allgather_and_scatter_are_message_for_message():
    """After the lane reduction the reference posts its bcast + Bruck (allreduce) or k-nomial
    scatter (reduce-scatter) and nothing else, so those are the last messages of every rank's
    trace: the exact plan's messages of those phases must be the same multiset of
    (direction, peer, bytes), rank by rank.  C4 (n=8, k=4, b=4) is in the grid: nnodes = 2 < b
    makes its whole allgather the reference's left-over Bruck (:645-756)."""
    bad = []
    for c in _traces():
        mode = ca.MODE_ALLREDUCE if c["mode"] == "ar" else ca.MODE_REDUCE_SCATTER
        for r in range(c["n"]):
            mine = _tail_messages(mode, c["n"], c["k"], c["b"], c["count"], r)
            ref = sorted(tuple(m) for m in c["ranks"][r][len(c["ranks"][r]) - len(mine):]) if mine else []
            if mine != ref:
                bad.append((c["mode"], c["n"], c["k"], c["b"], r))
    assert not bad, f"{len(bad)} ranks differ, e.g. {bad[:6]}"


def _inputs(c):
    n = c["n"]
    in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
    return [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]


def test_exact_plans_match_reference_golden(golden):
    cases, _ = golden
    bad, ran = [], 0
    for c in cases:
        if c["mode"] == "ag" or c["count"] * c["n"] > (1 << 16):
            continue
        mode = ca.MODE_ALLREDUCE if c["mode"] == "ar" else ca.MODE_REDUCE_SCATTER
        outs = plan_sim.simulate(mode, _inputs(c), c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]),
                                 schedule=ca.SCHEDULE_EXACT)
        ran += 1
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert ran > 500
    assert not bad, f"{len(bad)} exact-plan/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 8), (16, 4, 4), (24, 3, 4), (12, 5, 6), (27, 3, 3), (32, 2, 4)])
def test_exact_wider_grid(n, k, b):
    cnt = n * 5
    sends = [po.fill(cnt, "f32", 0, 91, r) for r in range(n)]
    ref = po.allreduce_radix_batch(sends, k, b, "f32", "sum")
    got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, k, b, "f32", "sum", schedule=ca.SCHEDULE_EXACT)
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), ref[r].view(np.uint32))
    sends = [po.fill(cnt, "f32", 0, 92, r) for r in range(n)]
    ref = po.reduce_scatter_radix_batch(sends, k, b, "f32", "sum")
    got = plan_sim.simulate(ca.MODE_REDUCE_SCATTER, sends, k, b, "f32", "sum", schedule=ca.SCHEDULE_EXACT)
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), ref[r].view(np.uint32))
