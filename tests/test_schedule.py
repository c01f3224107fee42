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
    in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
    return [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]


def test_plans_match_reference_golden(golden):
    cases, _ = golden
    bad = []
    for c in cases:
        if c["count"] * c["n"] > (1 << 16):
            continue  # the large hash-only cases are covered on the GPU
        mode = {"ar": ca.MODE_ALLREDUCE, "rs": ca.MODE_REDUCE_SCATTER, "ag": ca.MODE_ALLGATHER}[c["mode"]]
        outs = plan_sim.simulate(mode, _inputs(c), c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
        h = hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()
        if h != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} plan/reference mismatches, e.g. {bad[:5]}"


def test_one_shot_plans_match_reference_golden(golden):
    """SCHEDULE_FLAT_1SHOT (every rank receives the whole buffer from every peer and evaluates
    every chunk's tree itself): every golden case, pipelined at depth 2, bit-exact."""
    cases, _ = golden
    bad = []
    for c in cases:
        if c["count"] * c["n"] > (1 << 16):
            continue
        mode = {"ar": ca.MODE_ALLREDUCE, "rs": ca.MODE_REDUCE_SCATTER, "ag": ca.MODE_ALLGATHER}[c["mode"]]
        if mode == ca.MODE_ALLGATHER:
            continue
        outs = plan_sim.simulate(mode, _inputs(c), c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]), slices=2,
                                 schedule=ca.SCHEDULE_FLAT_1SHOT)
        h = hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()
        if h != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} one-shot plan/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 2), (8, 4, 8), (4, 4, 4), (2, 2, 2), (6, 2, 3), (16, 4, 4)])
def test_one_shot_plan_shape_and_traffic(n, k, b):
    """One exchange step per slice and no allgather: each rank sends its whole buffer to every peer,
    (n-1)·S bytes, against 2(n-1)/n·S for FLAT; the reduce-scatter plan is FLAT's."""
    count = n * 4096
    for rank in range(n):
        p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, n, rank, k, b, count, 3, ca.SCHEDULE_FLAT_1SHOT))
        assert p["header"]["schedule"] == ca.SCHEDULE_FLAT_1SHOT and p["header"]["steps"] == 3
        sent = sum(cnt for st in p["steps"] for _, _, cnt in st["sends"])
        assert sent == (n - 1) * count
        for st in p["steps"]:
            assert {peer for peer, _, _ in st["sends"]} == set(range(n)) - {rank}
        f = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, n, rank, k, b, count, 3, ca.SCHEDULE_FLAT))
        flat_sent = sum(cnt for st in f["steps"] for _, _, cnt in st["sends"])  # pieces are 64-element cuts
        assert abs(flat_sent - 2 * (n - 1) * count // n) <= 2 * n * 64 * 3 * (n // b)
        rs1 = ca.describe_plan(ca.MODE_REDUCE_SCATTER, n, rank, k, b, 4096, 2, ca.SCHEDULE_FLAT_1SHOT)
        rsf = ca.describe_plan(ca.MODE_REDUCE_SCATTER, n, rank, k, b, 4096, 2, ca.SCHEDULE_FLAT)
        assert rs1 == rsf


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
    one fused 3-input reduction per active lane, 1-input lane reduction at the roots,
    then the link-balanced distribute (scatter 1/7 pieces, forward).  Owner-lane evaluation
    (balance off)."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 20, schedule=ca.SCHEDULE_REFERENCE))
    assert p["header"]["k"] == 4 and p["header"]["steps"] == 4 and p["header"]["slices"] == 1
    ph = p["steps"][0]
    assert len(ph["recvs"]) == 3 and len(ph["sends"]) == 1
    red = [op for op in ph["post"] if op[0] == "reduce"]
    assert len(red) == 1 and len(red[0][4]) == 3
    lane = p["steps"][1]
    assert len(lane["recvs"]) == 1 and lane["post"][0][0] == "reduce"
    d1, d2 = p["steps"][2], p["steps"][3]
    assert len(d1["sends"]) == 7 and len(d1["recvs"]) == 1   # rank 0 owns chunk 0, gets a piece of chunk 1
    assert len(d2["sends"]) == 6 and len(d2["recvs"]) == 6  # forwards its piece of chunk 1, gets the rest


def test_plan_shape_c4_balanced():
    """Balanced C4: 3 steps; every rank exchanges with its 3 group peers (2 chunks each),
    reduces 2 chunks x 3 inputs, then 1 piece per chunk with the other node, then allgathers."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 5, 4, 4, 1 << 20, schedule=ca.SCHEDULE_BALANCED))
    assert p["header"]["balanced"] == 1 and p["header"]["steps"] == 3
    ph, lane, dist = p["steps"]
    assert len(ph["sends"]) == 6 and len(ph["recvs"]) == 6
    assert [len(op[4]) for op in ph["post"]] == [3, 3]
    assert {x[0] for x in lane["sends"]} == {1} and [len(op[4]) for op in lane["post"]] == [1, 1]
    assert all(op[1][0] == "RECV" for op in lane["post"])
    assert len(dist["sends"]) == 14 and len(dist["recvs"]) == 14


@pytest.mark.parametrize("slices", [2, 3, 5, 8])
@pytest.mark.parametrize("mode,n,k,b", [("ar", 8, 4, 4), ("ar", 8, 2, 2), ("ar", 8, 3, 4), ("ar", 12, 3, 6),
                                         ("ar", 2, 2, 1), ("rs", 8, 4, 4), ("rs", 2, 2, 2), ("rs", 12, 5, 6),
                                         ("ar", 16, 4, 8), ("ar", 9, 2, 3)])
def test_pipelined_plans_bit_exact(mode, n, k, b, slices):
    """Wavefront super-steps over element slices: same bits as the unsliced reference."""
    per = 256 * 5 + 64  # several 256-element slice granules per chunk, ragged last slice
    count = per * n
    m = ca.MODE_ALLREDUCE if mode == "ar" else ca.MODE_REDUCE_SCATTER
    in_n = count if mode == "ar" else count * n
    for dt in ("f32", "bf16"):
        sends = [po.fill(in_n, dt, 0, 314, r) for r in range(n)]
        f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
        ref = f(sends, k, b, dt, "sum")
        got = plan_sim.simulate(m, sends, k, b, dt, "sum", slices=slices)
        for r in range(n):
            np.testing.assert_array_equal(got[r], ref[r])


def test_pipelined_plan_structure():
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 8 * 4 * 4096, 4, schedule=ca.SCHEDULE_REFERENCE))
    assert p["header"]["slices"] == 4 and p["header"]["steps"] == 4 + 4 - 1
    # super-step 1 holds slice 0's lane reduce and slice 1's recexch phase in ONE group
    assert "lane/s0" in p["steps"][1]["label"] and "phase0/s1" in p["steps"][1]["label"]
    q = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 8 * 4 * 4096, 4, schedule=ca.SCHEDULE_BALANCED))
    assert q["header"]["steps"] == 3 + 4 - 1
    assert "blane/s0" in q["steps"][1]["label"] and "bphase/s1" in q["steps"][1]["label"]


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 8), (16, 3, 4), (6, 5, 3), (12, 8, 2), (1, 2, 1)])
def test_allgather_plans(n, k, b):
    """k-port direct allgather: in place and not, every rank gets the rank-major concatenation,
    k-1 peers per step, group peers first, each peer exactly once."""
    sends = [po.fill(11, "f32", po.PAT_UNIFORM, 3, r) for r in range(n)]
    want = po.allgather_radix_batch(sends, k, b, "f32")
    for inplace in (False, True):
        got = plan_sim.simulate(ca.MODE_ALLGATHER, sends, k, b, "f32", "sum", inplace=inplace)
        for r in range(n):
            np.testing.assert_array_equal(got[r], want[r])
    plans = plan_sim.load_plans(ca.MODE_ALLGATHER, n, k, b, 11)
    for r, p in enumerate(plans):
        peers = [x[0] for st in p["steps"] for x in st["sends"]]
        assert sorted(peers) == [q for q in range(n) if q != r]
        assert all(len(st["sends"]) <= k - 1 for st in p["steps"])
        assert set(peers[:b - 1]) == {q for q in range(r // b * b, r // b * b + b) if q != r}


def test_allgather_plan_errors():
    assert plan_sim.load_plans(ca.MODE_ALLGATHER, 6, 2, 4, 8)[0]["header"]["error"] == 3
    assert plan_sim.load_plans(ca.MODE_ALLGATHER, 6, 1, 3, 8)[0]["header"]["error"] == 1


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 2), (8, 8, 8), (8, 2, 1), (4, 4, 4), (2, 2, 2), (2, 2, 1),
                                   (6, 3, 3), (12, 4, 4), (16, 4, 4), (9, 3, 3), (5, 2, 1)])
@pytest.mark.parametrize("slices", [1, 3])
def test_balanced_plans_bit_exact(n, k, b, slices):
    """Balanced evaluation (every rank reduces 1/n of every chunk, same expressions) gives
    the reference's bits, with and without pipelining, for SUM and the order-sensitive MAX."""
    count = n * 1000 + n * 64
    for dt, op, pat in (("f32", "sum", po.PAT_UNIFORM), ("bf16", "sum", po.PAT_UNIFORM), ("f32", "max", po.PAT_TIES)):
        sends = [po.fill(count, dt, pat, 17, r) for r in range(n)]
        want = po.allreduce_radix_batch(sends, k, b, dt, op)
        plans = plan_sim.load_plans(ca.MODE_ALLREDUCE, n, k, b, count, slices, schedule=ca.SCHEDULE_BALANCED)
        assert plans[0]["header"]["balanced"] == 1
        got = plan_sim.execute(plans, sends, dt, op)
        for r in range(n):
            np.testing.assert_array_equal(got[r].view(np.uint8), want[r].view(np.uint8))


def test_balance_only_where_single_phase():
    hdr = lambda n, k, b: plan_sim.load_plans(ca.MODE_ALLREDUCE, n, k, b, n * 256,
                                              schedule=ca.SCHEDULE_BALANCED)[0]["header"]["balanced"]
    assert hdr(8, 4, 4) == 1 and hdr(8, 8, 8) == 1 and hdr(8, 2, 1) == 1
    assert hdr(8, 2, 4) == 0 and hdr(8, 3, 4) == 0 and hdr(8, 4, 8) == 0  # multi-phase / fold
    rs = lambda k, b: plan_sim.load_plans(ca.MODE_REDUCE_SCATTER, 8, k, b, 256,
                                          schedule=ca.SCHEDULE_BALANCED)[0]["header"]["balanced"]
    assert rs(4, 4) == 1 and rs(2, 4) == 0


def _link_bytes(plans):
    per_pair = {}
    for r, p in enumerate(plans):
        for st in p["steps"]:
            for peer, _, cnt in st["sends"]:
                per_pair[(r, peer)] = per_pair.get((r, peer), 0) + cnt
    return per_pair


def test_balanced_traffic_c4():
    """C4 geometry (n=8, k=4, b=4): the same total bytes, every rank sending exactly the
    allreduce minimum 2(n-1)/n of the buffer, and the busiest directed link carrying S/4 + S/8
    instead of ~0.64 S."""
    n, count = 8, 8 * 4096
    bal = _link_bytes(plan_sim.load_plans(ca.MODE_ALLREDUCE, n, 4, 4, count, schedule=ca.SCHEDULE_BALANCED))
    ref = _link_bytes(plan_sim.load_plans(ca.MODE_ALLREDUCE, n, 4, 4, count, schedule=ca.SCHEDULE_REFERENCE))
    per_rank = lambda d, r: sum(v for (a, _), v in d.items() if a == r)
    assert sum(bal.values()) == sum(ref.values())
    for r in range(n):  # balanced: every rank sends exactly the allreduce minimum
        assert per_rank(bal, r) == 2 * (n - 1) * count // n
    assert max(bal.values()) <= count // 4 + count // 8 + 64
    assert max(ref.values()) > 0.6 * count


@pytest.mark.parametrize("n,k,b", [(2, 2, 2), (2, 2, 1), (8, 4, 4), (8, 8, 8), (8, 2, 1), (6, 3, 3), (12, 4, 4),
                                   (16, 2, 2)])
@pytest.mark.parametrize("slices", [1, 3])
def test_balanced_reduce_scatter_bit_exact(n, k, b, slices):
    """Balanced reduce-scatter: rank (Y, j) evaluates exactly its own output block (sub-block j
    of chunk Y) in the reference's operand order -- no scatter phase, same bits."""
    rc = 64 * 7 + 3
    for dt, op, pat in (("f32", "sum", po.PAT_UNIFORM), ("bf16", "sum", po.PAT_UNIFORM), ("f32", "max", po.PAT_TIES)):
        sends = [po.fill(rc * n, dt, pat, 9, r) for r in range(n)]
        want = po.reduce_scatter_radix_batch(sends, k, b, dt, op)
        got = plan_sim.simulate(ca.MODE_REDUCE_SCATTER, sends, k, b, dt, op, slices=slices,
                                schedule=ca.SCHEDULE_BALANCED)
        for r in range(n):
            np.testing.assert_array_equal(got[r].view(np.uint8), want[r].view(np.uint8))


def test_balanced_reduce_scatter_traffic_c3():
    """C3 (n=2, k=2, b=2): each rank sends exactly the reduce-scatter minimum (n-1)/n of its
    send buffer; the reference's lane 0 receives the whole buffer and scatters half back."""
    n, rc = 2, 4096
    bal = _link_bytes(plan_sim.load_plans(ca.MODE_REDUCE_SCATTER, n, 2, 2, rc, schedule=ca.SCHEDULE_BALANCED))
    ref = _link_bytes(plan_sim.load_plans(ca.MODE_REDUCE_SCATTER, n, 2, 2, rc, schedule=ca.SCHEDULE_REFERENCE))
    assert bal == {(0, 1): rc, (1, 0): rc}
    assert max(ref.values()) == 2 * rc and sum(ref.values()) == 3 * rc


@pytest.mark.parametrize("n,k,b", [(8, 4, 4), (8, 2, 4), (8, 3, 4), (8, 2, 2), (8, 4, 8), (8, 8, 8), (6, 5, 3),
                                   (12, 3, 6), (16, 4, 4), (2, 2, 1)])
def test_flat_traffic_is_full_mesh_optimal(n, k, b):
    """Flat schedule, any geometry (multi-phase, fold, clamped k): every directed pair carries
    2S/n (allreduce) or S/n (reduce-scatter) up to 64-element piece alignment, and the plan is
    two / one steps deep."""
    count = n * 64 * 64
    ar = plan_sim.load_plans(ca.MODE_ALLREDUCE, n, k, b, count, schedule=ca.SCHEDULE_FLAT)
    assert ar[0]["header"]["schedule"] == ca.SCHEDULE_FLAT and ar[0]["header"]["steps"] == 2
    pair = _link_bytes(ar)
    assert len(pair) == n * (n - 1)
    assert max(pair.values()) - min(pair.values()) <= 2 * 64 * (n // b + 1)
    assert sum(pair.values()) == 2 * (n - 1) * count
    rc = 64 * 64
    rs = plan_sim.load_plans(ca.MODE_REDUCE_SCATTER, n, k, b, rc, schedule=ca.SCHEDULE_FLAT)
    assert set(_link_bytes(rs).values()) == {rc}


@pytest.mark.parametrize("n,k,b", [(8, 2, 4), (8, 3, 4), (12, 3, 6), (9, 2, 3), (16, 4, 8), (6, 5, 3)])
def test_flat_multi_phase_and_fold_bit_exact(n, k, b):
    """Expression trees with several recexch phases and step-1 folds, evaluated by the flat
    schedule (pipelined, in place and not): the reference's bits."""
    count = n * 640
    for dt, op, pat in (("f32", "sum", po.PAT_UNIFORM), ("f32", "min", po.PAT_TIES), ("bf16", "sum", po.PAT_UNIFORM)):
        sends = [po.fill(count, dt, pat, 23, r) for r in range(n)]
        want = po.allreduce_radix_batch(sends, k, b, dt, op)
        for inplace in (False, True):
            got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, k, b, dt, op, inplace=inplace, slices=2,
                                    schedule=ca.SCHEDULE_FLAT)
            for r in range(n):
                np.testing.assert_array_equal(got[r].view(np.uint8), want[r].view(np.uint8))
        rsends = [po.fill(count, dt, pat, 24, r) for r in range(n)]
        rwant = po.reduce_scatter_radix_batch(rsends, k, b, dt, op)
        rgot = plan_sim.simulate(ca.MODE_REDUCE_SCATTER, rsends, k, b, dt, op, slices=2, schedule=ca.SCHEDULE_FLAT)
        for r in range(n):
            np.testing.assert_array_equal(rgot[r].view(np.uint8), rwant[r].view(np.uint8))


@pytest.mark.parametrize("schedule", [0, 1, 2])
@pytest.mark.parametrize("n,k,b", [(12, 2, 1), (16, 3, 1), (16, 16, 16), (12, 12, 12), (10, 2, 1)])
def test_wide_fan_in_in_place(schedule, n, k, b):
    """Reductions with more than 8 inputs chain through dst on the device; an input that aliases
    dst (the own leaf read in place) must be folded before dst is written (plans split such
    reductions through STAGE scratch; plan_sim models the launcher's chaining)."""
    count = n * 64
    for dt, op, pat in (("f32", "sum", po.PAT_UNIFORM), ("f32", "min", po.PAT_TIES)):
        sends = [po.fill(count, dt, pat, 31, r) for r in range(n)]
        want = po.allreduce_radix_batch(sends, k, b, dt, op)
        got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, k, b, dt, op, inplace=True, schedule=schedule)
        for r in range(n):
            np.testing.assert_array_equal(got[r].view(np.uint8), want[r].view(np.uint8))
        rs = [po.fill(count, dt, pat, 32, r) for r in range(n)]
        rwant = po.reduce_scatter_radix_batch(rs, k, b, dt, op)
        rgot = plan_sim.simulate(ca.MODE_REDUCE_SCATTER, rs, k, b, dt, op, inplace=True, schedule=schedule)
        for r in range(n):
            np.testing.assert_array_equal(rgot[r].view(np.uint8), rwant[r].view(np.uint8))


@pytest.mark.parametrize("algo,n,k", [("rx", 16, 13), ("rx", 12, 12), ("rm", 16, 16), ("rm", 12, 11),
                                      ("krsag", 16, 12)])
def test_wide_mpich_chains_in_place(algo, n, k):
    """MPICH_do_reduce / recursive multiplying fold recvbuf into chains of k-1 > 8 operands."""
    mode = {"rx": ca.MODE_MPICH_RECEXCH, "rm": ca.MODE_MPICH_RMULT, "krsag": ca.MODE_MPICH_KRSAG}[algo]
    count = 300
    for op, pat in (("sum", po.PAT_UNIFORM), ("max", po.PAT_TIES)):
        sends = [po.fill(count, "f32", pat, 33, r) for r in range(n)]
        want = po.mpich_allreduce(algo, sends, "f32", op, k=k)
        for inplace in (False, True):
            got = plan_sim.simulate(mode, sends, k, 0, "f32", op, inplace=inplace)
            for r in range(n):
                np.testing.assert_array_equal(got[r].view(np.uint8), want[r].view(np.uint8))


def test_flat_merged_groups_and_dependencies():
    """Default flat plan: one RCCL group per step holds the gather of slice t and the allgather
    of slice t-2 (P + 2 groups); each step waits exactly for the evaluation of slice t-2, which
    ran while step t-1 was on the links."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 24, 4))
    labels = [st["label"] for st in p["steps"]]
    assert labels == ["gather/s0", "gather/s1", "gather/s2,fdist/s0", "gather/s3,fdist/s1", "fdist/s2", "fdist/s3"]
    assert [st["wait"] for st in p["steps"]] == [-1, -1, 0, 1, 2, 3]


def test_flat_overlap_dependencies():
    """Two-stream execution: in the flat_seq plan (separate groups), gather s+1 never waits for
    the evaluation of slice s (overlap), while allgather s waits exactly for it; wavefront plans
    wait step to step."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 24, 4, ca.SCHEDULE_FLAT_SEQ))
    labels = [st["label"] for st in p["steps"]]
    assert labels == ["gather/s0", "gather/s1", "fdist/s0", "gather/s2", "fdist/s1", "gather/s3", "fdist/s2",
                      "fdist/s3"]
    waits = {st["label"]: st["wait"] for st in p["steps"]}
    assert all(waits[f"gather/s{s}"] == -1 for s in range(4))
    for s in range(4):
        assert labels[waits[f"fdist/s{s}"]] == f"gather/s{s}"
    r = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 24, 4, ca.SCHEDULE_REFERENCE))
    assert [st["wait"] for st in r["steps"]][1:6] == [0, 1, 2, 3, 4]


@pytest.mark.parametrize("n,k,b,dt,slices", [(8, 4, 4, "f32", 2), (8, 2, 8, "bf16", 3), (4, 4, 4, "f32", 1),
                                             (2, 2, 1, "f64", 2), (6, 2, 3, "f32", 1)])
def test_flat_rccl_allgather_variant(n, k, b, dt, slices):
    """SCHEDULE_FLAT_AG: the flat plan with its allgather phase as in-place ncclAllGather
    collectives (equal pieces) -- same bits as the oracle."""
    cnt = n * 64 * 8
    sends = [po.fill(cnt, dt, 0, 55, r) for r in range(n)]
    plans = plan_sim.load_plans(ca.MODE_ALLREDUCE, n, k, b, cnt, slices, schedule=ca.SCHEDULE_FLAT_AG)
    # slices whose pieces are equal use the collective (with 3 slices some are unequal: p2p)
    assert any(st["allgathers"] and not st["sends"] for st in plans[0]["steps"] if st["label"].startswith("fdist"))
    got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, k, b, dt, "sum", slices=slices, schedule=ca.SCHEDULE_FLAT_AG)
    ref = po.allreduce_radix_batch(sends, k, b, dt, "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint8), ref[r].view(np.uint8))


def test_flat_rccl_allgather_unequal_pieces_fall_back_to_p2p():
    n = 8
    cnt = n * 100  # irc pieces are not equal: that slice's allgather stays point-to-point
    plans = plan_sim.load_plans(ca.MODE_ALLREDUCE, n, 4, 4, cnt, 1, schedule=ca.SCHEDULE_FLAT_AG)
    assert not any(st["allgathers"] for st in plans[0]["steps"])
    sends = [po.fill(cnt, "f32", 0, 56, r) for r in range(n)]
    got = plan_sim.simulate(ca.MODE_ALLREDUCE, sends, 4, 4, "f32", "sum", schedule=ca.SCHEDULE_FLAT_AG)
    ref = po.allreduce_radix_batch(sends, 4, 4, "f32", "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), ref[r].view(np.uint32))


@pytest.mark.parametrize("schedule", [ca.SCHEDULE_REFERENCE, ca.SCHEDULE_BALANCED, ca.SCHEDULE_FLAT, ca.SCHEDULE_EXACT,
                                      ca.SCHEDULE_FLAT_AG, ca.SCHEDULE_FLAT_SEQ, ca.SCHEDULE_FLAT_1SHOT])
def test_tiny_and_ragged_sizes_every_schedule(schedule):
    """One element per rank, odd per-rank counts, reduce-scatter recvcount 1/3/5: plans of every
    schedule reproduce the oracle bit-exactly (the GPU twin is in test_gpu_collectives.py)."""
    for n, k, b in ((8, 4, 4), (8, 2, 8), (8, 3, 2), (6, 2, 3), (6, 4, 6)):
        for per in (1, 3, 5):
            for mode in (ca.MODE_ALLREDUCE, ca.MODE_REDUCE_SCATTER):
                count = per * n if mode == ca.MODE_ALLREDUCE else per
                in_n = count if mode == ca.MODE_ALLREDUCE else count * n
                sends = [po.fill(in_n, "f32", 0, 17, r) for r in range(n)]
                got = plan_sim.simulate(mode, sends, k, b, "f32", "sum", schedule=schedule)
                f = po.allreduce_radix_batch if mode == ca.MODE_ALLREDUCE else po.reduce_scatter_radix_batch
                want = f(sends, k, b, "f32", "sum")
                for r in range(n):
                    np.testing.assert_array_equal(got[r].view(np.uint32), want[r].view(np.uint32))


@pytest.mark.parametrize("schedule", [ca.SCHEDULE_FLAT, ca.SCHEDULE_EXACT, ca.SCHEDULE_REFERENCE,
                                      ca.SCHEDULE_FLAT_1SHOT])
def test_plans_match_pair_and_complex_goldens(golden_pairtypes, schedule):
    """MAXLOC / MINLOC on the pair types and complex SUM / PROD through the compiled plans (CPU plan
    interpreter): the radix/batch and allgather goldens bit-exact under three schedules -- the TIES
    pattern's -0 / +0 and NaN cases fix the operand order of every reduction."""
    cases, _ = golden_pairtypes
    bad, ran = [], 0
    for c in cases:
        mode = {"ar": "ar", "rs": "rs", "ag": "ag", "ar_lib": "ar", "rs_lib": "rs"}.get(c["mode"])
        if mode is None:
            continue
        mm = {"ar": ca.MODE_ALLREDUCE, "rs": ca.MODE_REDUCE_SCATTER, "ag": ca.MODE_ALLGATHER}[mode]
        outs = plan_sim.simulate(mm, _inputs(dict(c, mode=mode)), c["k"], c["b"], c["dtype"], c["op"],
                                 bool(c["inplace"]), schedule=schedule)
        ran += 1
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert ran > 400 and not bad, f"{len(bad)} plan/reference mismatches, e.g. {bad[:5]}"


def test_plan_dependency_lists():
    """Every step lists all earlier steps whose local ops conflict with its transfers (comm_deps, the
    last of which is comm_wait): the executor's transfer stream waits on the latest of them, and the
    one compute stream runs local ops in order.  Checked here on the flat C4 plan: the evaluation of
    slice s reads only slice s's receives, and allgather s depends on exactly the evaluation of slice s."""
    p = ca.parse_plan(ca.describe_plan(ca.MODE_ALLREDUCE, 8, 0, 4, 4, 1 << 24, 4))
    assert [st["wait"] for st in p["steps"]] == [-1, -1, 0, 1, 2, 3]
    assert [st["deps"] for st in p["steps"]] == [[], [], [0], [1], [2], [3]]
    for sched in (ca.SCHEDULE_REFERENCE, ca.SCHEDULE_EXACT):
        for mode, count in ((ca.MODE_ALLREDUCE, 1 << 20), (ca.MODE_REDUCE_SCATTER, 1 << 17)):
            for rank in range(8):
                q = ca.parse_plan(ca.describe_plan(mode, 8, rank, 4, 4, count, 2, sched))
                for t, st in enumerate(q["steps"]):
                    assert st["deps"] == sorted(st["deps"]) and all(d < t for d in st["deps"])
                    assert st["wait"] == (st["deps"][-1] if st["deps"] else -1)
                    assert all(q["steps"][d]["post"] for d in st["deps"])


def _regions(op):
    """(buffer space, lo, hi) read and written by one parsed local op; SEND and RECV share a space
    (MPI_IN_PLACE makes them the same memory)."""
    sp = lambda b: "RECV" if b == "SEND" else b  # noqa: E731
    kind = op[0]
    cnt = op[3]
    if kind == "copy2d":
        rows, dp, spp = op[4]
        return ([(sp(op[2][0]), op[2][1] + r * spp, op[2][1] + r * spp + cnt) for r in range(rows)],
                [(sp(op[1][0]), op[1][1] + r * dp, op[1][1] + r * dp + cnt) for r in range(rows)])
    rd = [(sp(op[2][0]), op[2][1], op[2][1] + cnt)] + [(sp(x[0]), x[1], x[1] + cnt) for x in op[4]] \
        if kind in ("reduce", "reduce_sw", "tree") else [(sp(op[2][0]), op[2][1], op[2][1] + cnt)]
    wr = [(sp(op[1][0]), op[1][1], op[1][1] + cnt)]
    return rd, wr


def test_plan_dependencies_cover_in_place_aliasing():
    """under CHR_IN_PLACE the SEND and RECV regions are one buffer.  For every schedule and
    a spread of geometries, a step's transfers must list (in deps) every earlier step whose local ops
    write memory those transfers read or write, or read memory they write -- with SEND and RECV
    compared in one address space.  Missing one would let the transfer stream race the compute stream."""
    bad = []
    for sched in (ca.SCHEDULE_REFERENCE, ca.SCHEDULE_BALANCED, ca.SCHEDULE_FLAT, ca.SCHEDULE_EXACT,
                  ca.SCHEDULE_FLAT_AG, ca.SCHEDULE_FLAT_SEQ):
        for mode, count in ((ca.MODE_ALLREDUCE, 3 << 12), (ca.MODE_REDUCE_SCATTER, 3 << 9)):
            for n, k, b in ((8, 4, 4), (8, 2, 2), (6, 3, 3), (4, 2, 4)):
                for rank in range(n):
                    q = ca.parse_plan(ca.describe_plan(mode, n, rank, k, b, count - count % n, 2, sched))
                    steps = q["steps"]
                    rw = []
                    for st in steps:
                        rd, wr = [], []
                        for op in st["post"]:
                            r_, w_ = _regions(op)
                            rd += r_
                            wr += w_
                        rw.append((rd, wr))
                    sp = lambda b_: "RECV" if b_ == "SEND" else b_  # noqa: E731
                    for t, st in enumerate(steps):
                        crd = [(sp(x[1][0]), x[1][1], x[1][1] + x[2]) for x in st["sends"]]
                        cwr = [(sp(x[1][0]), x[1][1], x[1][1] + x[2]) for x in st["recvs"]]
                        for u in range(t):
                            rd, wr = rw[u]
                            hit = any(a[0] == c[0] and a[1] < c[2] and c[1] < a[2]
                                      for a in wr for c in crd + cwr) or \
                                any(a[0] == c[0] and a[1] < c[2] and c[1] < a[2] for a in rd for c in cwr)
                            if hit and u not in st["deps"]:
                                bad.append((sched, mode, n, k, b, rank, t, u))
    assert not bad, bad[:5]
