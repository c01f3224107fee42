"""Whole radix/batch collectives on the GPU vs the reference's golden vectors and the oracle.

Multi-rank schedules run on ONE MI355X through the loopback transport (LocalGroup):
the same compiled plans and the same HIP reduction kernels as the RCCL path, with
messages as device copies.  The RCCL path itself is exercised at nranks=1 here (the
box has one GPU) and at 2/4/8 GPUs by bench.py on the driver's 8-GPU node."""
import hashlib

import numpy as np
import pytest

import chiara_amd as ca
import pyoracle as po

pytestmark = pytest.mark.gpu

DT = {"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32, "bf16": ca.BFLOAT16, "i8": ca.INT8, "u8": ca.UINT8,
      "i16": ca.INT16, "u16": ca.UINT16, "u32": ca.UINT32, "i64": ca.INT64, "u64": ca.UINT64,
      "fi": ca.FLOAT_INT, "di": ca.DOUBLE_INT, "li": ca.LONG_INT, "2i": ca.TWO_INT, "si": ca.SHORT_INT,
      "cf": ca.C_FLOAT_COMPLEX, "cd": ca.C_DOUBLE_COMPLEX}
SCHEDULES = {"flat": ca.SCHEDULE_FLAT, "balanced": ca.SCHEDULE_BALANCED, "reference": ca.SCHEDULE_REFERENCE,
             "exact": ca.SCHEDULE_EXACT, "flat_ag": ca.SCHEDULE_FLAT_AG, "flat_seq": ca.SCHEDULE_FLAT_SEQ,
             "flat_1shot": ca.SCHEDULE_FLAT_1SHOT}
OP = {"sum": ca.SUM, "prod": ca.PROD, "max": ca.MAX, "min": ca.MIN, "land": ca.LAND, "lor": ca.LOR,
      "lxor": ca.LXOR, "band": ca.BAND, "bor": ca.BOR, "bxor": ca.BXOR, "maxloc": ca.MAXLOC, "minloc": ca.MINLOC}


@pytest.fixture(scope="module")
def gu():
    import gpu_util

    return gpu_util


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


def run_local(gu, group, mode, sends, k, b, dtype, op, inplace=False):
    n = len(sends)
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    count = sends[0].size // n if mode == "rs" else sends[0].size
    outc = count * n if mode == "ag" else count
    if mode == "ag":
        d_recv = [gu.empty_dev(outc * es) for _ in range(n)]
        if inplace:
            for r in range(n):
                d_recv[r][r * count * es:(r + 1) * count * es].copy_(gu.to_dev(sends[r]))
            d_sendp = [ca.IN_PLACE] * n
        else:
            d_sendp = [gu.to_dev(s) for s in sends]
        rc = group.allgather_radix_batch(d_sendp, count, DT[dtype], d_recv, k, b)
        assert rc == 0, f"rc={rc}"
        return [gu.from_dev(d, npdt, outc) for d in d_recv]
    d_send = [gu.to_dev(s) for s in sends]
    if inplace:
        d_recv, d_sendp = d_send, [ca.IN_PLACE] * n
    else:
        d_recv = [gu.empty_dev(count * es) for _ in range(n)]
        d_sendp = d_send
    fn = group.all_reduce_radix_batch if mode == "ar" else group.reduce_scatter_radix_batch
    rc = fn(d_sendp, d_recv, count, DT[dtype], OP[op], k, b)
    assert rc == 0, f"rc={rc}"
    return [gu.from_dev(d, npdt, outc) for d in d_recv]


def test_local_group_matches_reference_golden(gu, groups, golden):
    """Every golden case (1000+ geometries/dtypes/ops/in-place) bit-exact on the device."""
    cases, _ = golden
    bad = []
    for c in cases:
        n = c["n"]
        in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
        sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        outs = run_local(gu, groups(n), c["mode"], sends, c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
        h = hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()
        if h != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("schedule", ["exact", "flat_1shot"])
def test_local_group_exact_schedule_matches_reference_golden(gu, groups, golden, schedule):
    """The exact schedule (reference messages end to end) and the one-shot flat schedule (every rank
    evaluates the whole buffer) on the device, every radix/batch golden case."""
    cases, _ = golden
    bad = []
    for c in cases:
        if c["mode"] == "ag":
            continue
        n = c["n"]
        in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
        sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        g = groups(n)
        g.set_schedule(SCHEDULES[schedule])
        try:
            outs = run_local(gu, g, c["mode"], sends, c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
        finally:
            g.set_schedule(ca.SCHEDULE_FLAT)
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


def _golden_on_device(gu, groups, c, schedule):
    """One golden case through the local group: the radix/batch collectives (ar_lib / rs_lib: the
    same calls, compared with MPI's own collective) or an MPICH baseline; every rank's output."""
    n, g = c["n"], groups(c["n"])
    mode = {"ar_lib": "ar", "rs_lib": "rs"}.get(c["mode"], c["mode"])
    if mode in ("ar", "rs", "ag"):
        in_n = c["count"] * n if mode == "rs" else c["count"]
        sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        g.set_schedule(ca.SCHEDULE_EXACT if schedule == "exact" else ca.SCHEDULE_FLAT)
        try:
            return run_local(gu, g, mode, sends, c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
        finally:
            g.set_schedule(ca.SCHEDULE_FLAT)
    npdt = po.NP_DTYPES[c["dtype"]]
    sends = [po.fill(c["count"], c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
    d_send = [gu.to_dev(x) for x in sends]
    if c["inplace"]:
        d_recv, d_sendp = d_send, [ca.IN_PLACE] * n
    else:
        d_recv, d_sendp = [gu.empty_dev(x.nbytes) for x in sends], d_send
    assert g.allreduce_mpich(MPICH_MODE[mode], d_sendp, d_recv, c["count"], DT[c["dtype"]], OP[c["op"]],
                             c["k"], c["b"]) == 0, c["id"]
    return [gu.from_dev(d, npdt, c["count"]) for d in d_recv]


@pytest.mark.parametrize("schedule", ["flat", "exact"])
def test_pair_and_complex_types_match_reference_golden(gu, groups, golden_pairtypes, schedule):
    """MPI_MAXLOC / MPI_MINLOC on the five pair types and SUM / PROD on the C complex types (the
    reference's generic MPI_Datatype x MPI_Op, all_reduce_radix_batch.cpp:202-204): every golden
    case bit-exact on the device -- the reference run here under MPICH 3.3.2 for MPI_FLOAT_INT,
    MPI_2INT and complex (the TIES pattern's -0 / +0 and NaN expose the operand order), MPI's own
    collective for the types the reference mis-strides (gen_golden.py pairs_cases_for)."""
    cases, _ = golden_pairtypes
    bad = []
    for c in cases:
        if schedule == "exact" and c["mode"] not in ("ar", "rs", "ar_lib", "rs_lib"):
            continue
        outs = _golden_on_device(gu, groups, c, schedule)
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("schedule", ["flat", "exact"])
def test_integer_types_and_logical_bitwise_ops_match_reference_golden(gu, groups, golden_types, schedule):
    """The reference's generic MPI_Datatype x MPI_Op (all_reduce_radix_batch.cpp:202-204,
    :234-277): (u)int8/16/64, uint32 and LAND/LOR/LXOR/BAND/BOR/BXOR through the radix/batch
    collectives and the MPICH baselines, every golden case of the reference run under MPICH 3.3.2
    bit-exact on the device."""
    cases, _ = golden_types
    bad = []
    for c in cases:
        if schedule == "exact" and c["mode"] not in ("ar", "rs"):
            continue
        n, g = c["n"], groups(c["n"])
        if c["mode"] in ("ar", "rs", "ag"):
            in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
            sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
            g.set_schedule(ca.SCHEDULE_EXACT if schedule == "exact" else ca.SCHEDULE_FLAT)
            try:
                outs = run_local(gu, g, c["mode"], sends, c["k"], c["b"], c["dtype"], c["op"], bool(c["inplace"]))
            finally:
                g.set_schedule(ca.SCHEDULE_FLAT)
        else:
            npdt = po.NP_DTYPES[c["dtype"]]
            sends = [po.fill(c["count"], c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
            d_send = [gu.to_dev(x) for x in sends]
            if c["inplace"]:
                d_recv, d_sendp = d_send, [ca.IN_PLACE] * n
            else:
                d_recv, d_sendp = [gu.empty_dev(x.nbytes) for x in sends], d_send
            assert g.allreduce_mpich(MPICH_MODE[c["mode"]], d_sendp, d_recv, c["count"], DT[c["dtype"]], OP[c["op"]],
                                     c["k"], c["b"]) == 0, c["id"]
            outs = [gu.from_dev(d, npdt, c["count"]) for d in d_recv]
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("mode,n,k,b,dtype", [
    ("ar", 8, 4, 4, "f32"), ("ar", 8, 4, 4, "bf16"), ("ar", 8, 2, 2, "f32"), ("ar", 8, 3, 4, "bf16"),
    ("ar", 8, 2, 4, "bf16"), ("ar", 8, 4, 8, "f32"), ("rs", 2, 2, 1, "f32"), ("rs", 2, 2, 2, "f32"),
    ("ar", 2, 2, 1, "f32"), ("ar", 2, 2, 2, "f32"), ("ar", 16, 4, 4, "f32"), ("rs", 8, 4, 4, "bf16"),
])
@pytest.mark.parametrize("slices", [1, 3, 8])
def test_baseline_geometries_vs_oracle(gu, groups, mode, n, k, b, dtype, slices):
    """BASELINE configs' (n, k, b) at 4-16 MiB per rank, unsliced and pipelined: bit-exact vs the oracle."""
    per_rank = (1 << 22) if dtype == "f32" else (1 << 23)
    in_n = per_rank if mode == "ar" else per_rank // n * n
    sends = [po.fill(in_n, dtype, 0, 0xC41A5EED, r) for r in range(n)]
    g = groups(n)
    g.set_slices(slices)
    try:
        got = run_local(gu, g, mode, sends, k, b, dtype, "sum")
    finally:
        g.set_slices(0)
    f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
    ref = f(sends, k, b, dtype, "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r], ref[r])


@pytest.mark.parametrize("schedule", ["flat", "exact", "flat_ag", "reference"])
def test_c4_full_size_exact_int(gu, groups, schedule):
    """C4 at full size (1 GiB per rank, 8 ranks, k=4, b=4) with the reference harness's
    int32 pattern rank*count+i: every rank must hold sum_r (r*count + i) exactly, under the
    default schedule and the reference-message (exact), RCCL-allgather and reference routes."""
    import torch

    n, k, b, count = 8, 4, 4, 1 << 28
    g = groups(n)
    sends = [torch.empty(count, dtype=torch.int32, device=gu.DEV) for _ in range(n)]
    for r, s in enumerate(sends):
        assert ca.fill(s, count, ca.INT32, 1, 0, r, count, gu.stream()) == 0
    recvs = [torch.empty(count, dtype=torch.int32, device=gu.DEV) for _ in range(n)]
    gu.sync()
    g.set_schedule({"flat": ca.SCHEDULE_FLAT, "exact": ca.SCHEDULE_EXACT, "flat_ag": ca.SCHEDULE_FLAT_AG,
                    "reference": ca.SCHEDULE_REFERENCE}[schedule])
    try:
        assert g.all_reduce_radix_batch(sends, recvs, count, ca.INT32, ca.SUM, k, b) == 0
    finally:
        g.set_schedule(ca.SCHEDULE_FLAT)
    i = torch.arange(count, dtype=torch.int64, device=gu.DEV)
    expect = ((count * (n * (n - 1) // 2) + n * i) & 0xFFFFFFFF).to(torch.int64)
    expect = torch.where(expect >= 2**31, expect - 2**32, expect).to(torch.int32)
    for r in range(n):
        assert torch.equal(recvs[r], expect), f"rank {r}"
    del sends, recvs, i, expect
    torch.cuda.empty_cache()


@pytest.mark.parametrize("b", [1, 2])
def test_c3_full_size_bit_exact(gu, groups, b):
    """C3 at full size: reduce-scatter, n=2, k=2, recvcount 2^25 fp32 (256 MiB send buffer per
    rank), b in {1, 2}: bit-exact vs the oracle (fp32 data, U[-1,1))."""
    n, k, recvcount = 2, 2, 1 << 25
    sends = [po.fill(recvcount * n, "f32", po.PAT_UNIFORM, 0xC41A5EED, r) for r in range(n)]
    got = run_local(gu, groups(n), "rs", sends, k, b, "f32", "sum")
    ref = po.reduce_scatter_radix_batch(sends, k, b, "f32", "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), ref[r].view(np.uint32))


def test_c5_full_size_bf16_properties(gu, groups):
    """C5 geometry at full size (1 GiB bf16 per rank, 8 ranks, b=4, k=4): all ranks
    bit-identical, and within (n-1) bf16 ulps of the fp32 sum of the inputs."""
    import torch

    n, k, b, count = 8, 4, 4, 1 << 29
    g = groups(n)
    sends = [torch.empty(count, dtype=torch.bfloat16, device=gu.DEV) for _ in range(n)]
    for r, s in enumerate(sends):
        assert ca.fill(s, count, ca.BFLOAT16, 0, 0xC41A5EED, r, count, gu.stream()) == 0
    recvs = [torch.empty(count, dtype=torch.bfloat16, device=gu.DEV) for _ in range(n)]
    gu.sync()
    assert g.all_reduce_radix_batch(sends, recvs, count, ca.BFLOAT16, ca.SUM, k, b) == 0
    for r in range(1, n):
        assert torch.equal(recvs[r].view(torch.int16), recvs[0].view(torch.int16))
    step = 1 << 24
    for s0 in range(0, count, step):
        exact = sum(x[s0:s0 + step].float() for x in sends)
        bound = (n - 1) * 2.0 ** -8 * sum(x[s0:s0 + step].float().abs() for x in sends) + 1e-30
        assert bool(((recvs[0][s0:s0 + step].float() - exact).abs() <= bound).all())
    del sends, recvs
    torch.cuda.empty_cache()


SEED = 0xC41A5EED


def _window_reader(recvs, n, rc, npdt, tview):
    def out_window(r, off, w):
        return recvs[r].view(tview).view(n, rc)[:, off:off + w].contiguous().cpu().numpy().ravel().view(npdt)
    return out_window


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dtype,schedule,slices", [("f32", "flat", 0), ("f32", "flat", 8), ("f32", "exact", 0),
                                                   ("bf16", "flat", 0), ("bf16", "flat", 8), ("bf16", "exact", 0)])
def test_c4_c5_full_size_bit_exact_vs_oracle(gu, groups, dtype, schedule, slices):
    """C4 (fp32) and C5 (bf16) at their BASELINE size -- 8 ranks, k=4, b=4, 1 GiB per rank,
    U[-1,1) data -- bit-exact vs the C oracle over every element of every rank.  This is the
    size that switches on the non-temporal / ACC0 / one-wave kernel instantiations, the batched
    tree launches and the pipeline (automatic depth: 4 slices for flat, 16 MiB pieces; and 8);
    the association order the oracle pins is
    all_reduce_radix_batch.cpp:343-364 (recexch folds) and :523-530 (lane reduction).  The int32
    closed form (test_c4_full_size_exact_int) and the bf16 bound stay as fast pre-checks: both
    are blind to association.  Checked window by window (tests/fullsize_util.py)."""
    import torch

    import fullsize_util as fs

    n, k, b = 8, 4, 4
    es = 4 if dtype == "f32" else 2
    count = (1 << 30) // es
    rc = count // n
    cdt = DT[dtype]
    g = groups(n)
    sends = [torch.empty(count * es, dtype=torch.uint8, device=gu.DEV) for _ in range(n)]
    for r, s in enumerate(sends):
        assert ca.fill(s, count, cdt, po.PAT_UNIFORM, SEED, r, count, gu.stream()) == 0
    recvs = [torch.empty(count * es, dtype=torch.uint8, device=gu.DEV) for _ in range(n)]
    gu.sync()
    g.set_schedule({"flat": ca.SCHEDULE_FLAT, "exact": ca.SCHEDULE_EXACT}[schedule])
    g.set_slices(slices)
    try:
        assert g.all_reduce_radix_batch(sends, recvs, count, cdt, ca.SUM, k, b) == 0
    finally:
        g.set_schedule(ca.SCHEDULE_FLAT)
        g.set_slices(0)
    gu.sync()
    del sends
    torch.cuda.empty_cache()
    tview = torch.int32 if dtype == "f32" else torch.int16
    bad = fs.check_allreduce(_window_reader(recvs, n, rc, po.NP_DTYPES[dtype], tview), n, k, b, dtype, count, SEED)
    assert not bad, f"{len(bad)} (rank, window) mismatches vs the oracle, e.g. {bad[:5]}"
    del recvs
    torch.cuda.empty_cache()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("b", [1, 2])
def test_c3_full_size_windowed_inputs_from_device(gu, groups, b):
    """C3 (reduce-scatter, n=2, k=2, 256 MiB send buffer) with device-generated inputs, checked
    window by window like C4/C5: the windowed oracle path on a shape the whole-buffer oracle
    also covers (test_c3_full_size_bit_exact)."""
    import torch

    import fullsize_util as fs

    n, k, recvcount = 2, 2, 1 << 25
    sends = [torch.empty(recvcount * n * 4, dtype=torch.uint8, device=gu.DEV) for _ in range(n)]
    for r, s in enumerate(sends):
        assert ca.fill(s, recvcount * n, ca.FLOAT32, po.PAT_UNIFORM, SEED, r, recvcount * n, gu.stream()) == 0
    recvs = [torch.empty(recvcount * 4, dtype=torch.uint8, device=gu.DEV) for _ in range(n)]
    gu.sync()
    assert groups(n).reduce_scatter_radix_batch(sends, recvs, recvcount, ca.FLOAT32, ca.SUM, k, b) == 0
    gu.sync()

    def out_window(r, off, w):
        return recvs[r].view(torch.int32)[off:off + w].cpu().numpy().view(np.float32)
    bad = fs.check_reduce_scatter(out_window, n, k, b, "f32", recvcount, SEED)
    assert not bad, bad[:5]


def test_preconditions_rejected(gu, groups):
    g = groups(8)
    d = [gu.empty_dev(131 * 4) for _ in range(8)]
    assert g.all_reduce_radix_batch(d, d, 131, ca.FLOAT32, ca.SUM, 2, 2) == 2
    g6 = groups(6)
    d6 = [gu.empty_dev(24 * 4) for _ in range(6)]
    assert g6.all_reduce_radix_batch(d6, d6, 24, ca.FLOAT32, ca.SUM, 2, 4) == 3


def test_rccl_comm_single_rank(gu):
    """The RCCL transport end to end at nranks=1 (device and host buffers)."""
    import torch

    uid = ca.get_unique_id()
    comm = ca.Comm(1, uid, 0, 0)
    x = po.fill(4096, "f32", 0, 3, 0)
    ds, dr = gu.to_dev(x), gu.empty_dev(x.nbytes)
    assert ca.all_reduce_radix_batch(ds, dr, x.size, ca.FLOAT32, ca.SUM, comm, 2, 1) == 0
    np.testing.assert_array_equal(gu.from_dev(dr, np.float32), x)
    host_out = np.zeros_like(x)
    assert ca.all_reduce_radix_batch(x, host_out, x.size, ca.FLOAT32, ca.SUM, comm, 2, 1) == 0
    np.testing.assert_array_equal(host_out, x)
    assert ca.reduce_scatter_radix_batch(ds, dr, x.size, ca.FLOAT32, ca.SUM, comm, 2, 1) == 0
    np.testing.assert_array_equal(gu.from_dev(dr, np.float32), x)
    # a fixed schedule's (schedule, depth) for a call with these arguments -- and none for arguments such a call
    # rejects, or on an aborted communicator; the overlap setting read back from the library
    comm.set_schedule(ca.SCHEDULE_FLAT)
    assert comm.tuned_schedule(ca.MODE_ALLREDUCE, x.size, ca.FLOAT32, 2, 1) == (ca.SCHEDULE_FLAT, 1)
    assert comm.tuned_schedule(ca.MODE_ALLREDUCE, x.size, ca.FLOAT32, 1, 1) is None  # k < 2
    assert comm.tuned_schedule(ca.MODE_ALLREDUCE, x.size, ca.FLOAT32, 2, 3) is None  # nranks % b
    assert comm.tuned_schedule(5, x.size, ca.FLOAT32, 2, 1) is None  # not allreduce / reduce-scatter
    assert comm.overlap is True
    comm.set_overlap(False)
    assert comm.overlap is False
    comm.abort()
    assert comm.tuned_schedule(ca.MODE_ALLREDUCE, x.size, ca.FLOAT32, 2, 1) is None
    comm.destroy()
    torch.cuda.synchronize()


# ---- MPICH baselines (testing/main.cpp) on the same kernels --------------------------------

MPICH_MODE = {"ring": ca.MODE_MPICH_RING, "rd": ca.MODE_MPICH_RD, "rsag": ca.MODE_MPICH_RSAG,
              "rx": ca.MODE_MPICH_RECEXCH, "krsag": ca.MODE_MPICH_KRSAG, "rm": ca.MODE_MPICH_RMULT}


def test_mpich_baselines_match_reference_golden(gu, groups, golden_mpich):
    """All six testing/main.cpp baselines: every golden case bit-exact on the device."""
    cases, _ = golden_mpich
    bad = []
    for c in cases:
        n = c["n"]
        npdt = po.NP_DTYPES[c["dtype"]]
        sends = [po.fill(c["count"], c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        d_send = [gu.to_dev(s) for s in sends]
        if c["inplace"]:
            d_recv, d_sendp = d_send, [ca.IN_PLACE] * n
        else:
            d_recv, d_sendp = [gu.empty_dev(s.nbytes) for s in sends], d_send
        rc = groups(n).allreduce_mpich(MPICH_MODE[c["mode"]], d_sendp, d_recv, c["count"], DT[c["dtype"]],
                                       OP[c["op"]], c["k"], c["b"])
        assert rc == 0, (c["id"], rc)
        outs = [gu.from_dev(d, npdt, c["count"]) for d in d_recv]
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("algo", sorted(MPICH_MODE))
def test_mpich_baselines_large_int_exact(gu, groups, algo):
    """8 ranks, 4M int32 (the size class testing/main.cpp reaches): exact vs the oracle."""
    n, count = 8, (1 << 22) + 5
    sends = [po.fill(count, "i32", po.PAT_UNIFORM, 99, r) for r in range(n)]
    want = po.mpich_allreduce(algo, sends, "i32", "sum", k=3)
    d_send = [gu.to_dev(s) for s in sends]
    d_recv = [gu.empty_dev(s.nbytes) for s in sends]
    assert groups(n).allreduce_mpich(MPICH_MODE[algo], d_send, d_recv, count, ca.INT32, ca.SUM, 3, 0) == 0
    for r in range(n):
        np.testing.assert_array_equal(gu.from_dev(d_recv[r], np.int32, count), want[r])


@pytest.mark.parametrize("n,k,b,inplace", [(8, 4, 4, False), (8, 8, 8, True), (16, 3, 4, False), (6, 2, 3, True)])
def test_allgather_large_bit_exact(gu, groups, n, k, b, inplace):
    """allgather_radix_batch at 8 MiB per rank block: every byte in place."""
    count = (1 << 21) + 3
    sends = [po.fill(count, "f32", po.PAT_UNIFORM, 21, r) for r in range(n)]
    outs = run_local(gu, groups(n), "ag", sends, k, b, "f32", "sum", inplace)
    want = np.concatenate(sends)
    for r in range(n):
        np.testing.assert_array_equal(outs[r].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("n,k,b,dtype", [(8, 4, 4, "f32"), (8, 4, 4, "bf16"), (8, 8, 8, "f32"), (8, 2, 1, "f32"),
                                         (4, 4, 4, "f32"), (2, 2, 2, "f32")])
def test_schedules_bit_identical(gu, groups, n, k, b, dtype):
    """Flat, balanced, reference-communication and exact (the reference's messages end to end,
    unsliced) schedules, 8 MiB per rank: identical bits, all equal to the oracle."""
    count = (1 << 21) // (2 if dtype == "bf16" else 1) * 2
    count -= count % n
    sends = [po.fill(count, dtype, po.PAT_UNIFORM, 5, r) for r in range(n)]
    g = groups(n)
    outs = {}
    try:
        for sch in (ca.SCHEDULE_FLAT, ca.SCHEDULE_BALANCED, ca.SCHEDULE_REFERENCE, ca.SCHEDULE_EXACT,
                    ca.SCHEDULE_FLAT_AG, ca.SCHEDULE_FLAT_SEQ, ca.SCHEDULE_FLAT_1SHOT):
            g.set_schedule(sch)
            g.set_slices(3)
            outs[sch] = run_local(gu, g, "ar", sends, k, b, dtype, "sum")
    finally:
        g.set_schedule(ca.SCHEDULE_FLAT)
        g.set_slices(0)
    want = po.allreduce_radix_batch(sends, k, b, dtype, "sum")
    for r in range(n):
        for sch in outs:
            np.testing.assert_array_equal(outs[sch][r].view(np.uint8), want[r].view(np.uint8))


@pytest.mark.parametrize("n,k,b,dtype,slices,inplace", [(8, 4, 4, "f32", 0, False), (8, 4, 4, "bf16", 8, True),
                                                         (8, 2, 2, "f32", 3, False), (5, 2, 5, "i32", 2, True),
                                                         (4, 4, 4, "f64", 1, False)])
def test_local_group_cross_rank_batching_bit_identical(gu, groups, n, k, b, dtype, slices, inplace):
    """The virtual ranks' trees of one step share launches (chr_local_group_set_batching, default
    on) or run rank by rank: identical bits, equal to the oracle; allreduce (optionally in place,
    an odd per-rank count for scalar heads and tails) and reduce-scatter."""
    count = (3 << 20) + 8 * n + 5
    count -= count % n
    sends = [po.fill(count, dtype, po.PAT_UNIFORM, 9, r) for r in range(n)]
    g = groups(n)
    got = {}
    try:
        g.set_slices(slices)
        for on in (True, False):
            g.set_batching(on)
            got[on] = (run_local(gu, g, "ar", sends, k, b, dtype, "sum", inplace),
                       run_local(gu, g, "rs", sends, k, b, dtype, "sum"))
    finally:
        g.set_batching(True)
        g.set_slices(0)
    want_ar = po.allreduce_radix_batch(sends, k, b, dtype, "sum")
    want_rs = po.reduce_scatter_radix_batch(sends, k, b, dtype, "sum")
    for on in (True, False):
        for r in range(n):
            np.testing.assert_array_equal(got[on][0][r].view(np.uint8), want_ar[r].view(np.uint8))
            np.testing.assert_array_equal(got[on][1][r].view(np.uint8), want_rs[r].view(np.uint8))


@pytest.mark.parametrize("n,k,b", [(2, 2, 2), (2, 2, 1), (8, 4, 4), (8, 8, 8)])
def test_balanced_reduce_scatter_equals_owner_lane(gu, groups, n, k, b):
    """Reduce-scatter: balanced (own block evaluated locally) and owner-lane plans, 4 MiB
    blocks, both bit-exact vs the oracle."""
    rc = (1 << 20) + 64
    sends = [po.fill(rc * n, "f32", po.PAT_UNIFORM, 6, r) for r in range(n)]
    want = po.reduce_scatter_radix_batch(sends, k, b, "f32", "sum")
    g = groups(n)
    try:
        for sch in (ca.SCHEDULE_FLAT, ca.SCHEDULE_BALANCED, ca.SCHEDULE_REFERENCE, ca.SCHEDULE_EXACT):
            g.set_schedule(sch)
            got = run_local(gu, g, "rs", sends, k, b, "f32", "sum")
            for r in range(n):
                np.testing.assert_array_equal(got[r].view(np.uint32), want[r].view(np.uint32))
    finally:
        g.set_schedule(ca.SCHEDULE_FLAT)




@pytest.mark.parametrize("schedule", sorted(SCHEDULES))
def test_tiny_ragged_and_empty_every_schedule(gu, groups, schedule):
    """Edge sizes under every schedule: one element per rank, odd per-rank counts, reduce-scatter
    recvcount 1/3/5, and count 0 (a no-op returning success): bit-exact vs the oracle."""
    g8 = groups(8)
    g6 = groups(6)
    for g in (g8, g6):
        g.set_schedule(SCHEDULES[schedule])
    try:
        for n, g, k, b in ((8, g8, 4, 4), (8, g8, 2, 8), (8, g8, 3, 2), (6, g6, 2, 3), (6, g6, 4, 6)):
            for per in (1, 3, 5):
                for mode in ("ar", "rs"):
                    count = per * n if mode == "ar" else per
                    in_n = count if mode == "ar" else count * n
                    sends = [po.fill(in_n, "f32", 0, 17, r) for r in range(n)]
                    got = run_local(gu, g, mode, sends, k, b, "f32", "sum")
                    f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
                    want = f(sends, k, b, "f32", "sum")
                    for r in range(n):
                        np.testing.assert_array_equal(got[r].view(np.uint32), want[r].view(np.uint32))
            d = [gu.empty_dev(16) for _ in range(n)]
            assert g.all_reduce_radix_batch(d, d, 0, ca.FLOAT32, ca.SUM, k, b) == 0
            assert g.reduce_scatter_radix_batch(d, d, 0, ca.FLOAT32, ca.SUM, k, b) == 0
    finally:
        for g in (g8, g6):
            g.set_schedule(ca.SCHEDULE_FLAT)


RS_MODE = {"rs_radix": ca.MODE_MPICH_RS_RADIX, "rs_halving": ca.MODE_MPICH_RS_HALVING,
           "rs_doubling": ca.MODE_MPICH_RS_DOUBLING, "rs_pairwise": ca.MODE_MPICH_RS_PAIRWISE}


def test_mpich_reduce_scatter_baselines_match_reference_golden(gu, groups, golden_rsmpich):
    """The four baselines testing/mpich_implementations/reduce_scatter/main.cpp times (radix,
    recursive halving, recursive doubling with relays, pairwise): every golden case of the
    reference's own code bit-exact on the device, in place and not."""
    cases, _ = golden_rsmpich
    bad = []
    for c in cases:
        n = c["n"]
        npdt = po.NP_DTYPES[c["dtype"]]
        sends = [po.fill(c["count"] * n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        d_send = [gu.to_dev(x) for x in sends]
        if c["inplace"]:
            d_recv, d_sendp = d_send, [ca.IN_PLACE] * n
        else:
            d_recv, d_sendp = [gu.empty_dev(c["count"] * x.itemsize) for x in sends], d_send
        rc = groups(n).reduce_scatter_mpich(RS_MODE[c["mode"]], d_sendp, d_recv, c["count"], DT[c["dtype"]],
                                           OP[c["op"]], c["k"])
        assert rc == 0, (c["id"], rc)
        outs = [gu.from_dev(d, npdt, c["count"]) for d in d_recv]
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("algo", sorted(RS_MODE))
def test_mpich_reduce_scatter_baselines_large(gu, groups, algo):
    """6 ranks (non-power of two: folds and relays), 4 MiB fp32 blocks: bit-exact vs the oracle."""
    n, rc = 6, (1 << 20) + 3
    sends = [po.fill(rc * n, "f32", po.PAT_UNIFORM, 77, r) for r in range(n)]
    want = po.mpich_reduce_scatter(algo, sends, "f32", "sum", k=3)
    d_send = [gu.to_dev(x) for x in sends]
    d_recv = [gu.empty_dev(rc * 4) for _ in range(n)]
    assert groups(n).reduce_scatter_mpich(RS_MODE[algo], d_send, d_recv, rc, ca.FLOAT32, ca.SUM, 3) == 0
    for r in range(n):
        np.testing.assert_array_equal(gu.from_dev(d_recv[r], np.float32, rc).view(np.uint32), want[r].view(np.uint32))


PHASE_MODE = {"irs": ca.MODE_INTRA_REDUCE_SCATTER, "ilr": ca.MODE_INTER_REDUCE_LINEAR, "isc": ca.MODE_INTRA_SCATTER}


def _run_phase(gu, group, mode, sends, k, b, rc, dtype, op, inplace=False, null_unread=False):
    """Every rank's recv buffer after the stand-alone phase `mode` on the device (recv starts zero, so
    what a rank's plan does not write stays zero, as in the reference driver)."""
    n = len(sends)
    npdt = po.NP_DTYPES[dtype]
    in_n, out_n = po.phase_sizes(mode, n, b, rc)
    es = np.dtype(npdt).itemsize
    if inplace:
        d_recv = [gu.to_dev(s) for s in sends]
        d_sendp = [ca.IN_PLACE] * n
    else:
        d_recv = [gu.to_dev(np.zeros(max(out_n, 1), dtype=npdt)) for _ in range(n)]
        d_sendp = [gu.to_dev(s) for s in sends]
        if null_unread and mode == "isc":  # only node roots read their send buffer
            d_sendp = [d if (r % b) == (r // b) % b else None for r, d in enumerate(d_sendp)]
    d_recvp = list(d_recv)
    if null_unread and mode == "ilr" and not inplace:  # only the iterations' roots write recv
        nnodes = n // b
        for r in range(n):
            node, lane = divmod(r, b)
            if not any(i * b + lane == node for i in range(nnodes // b + (1 if nnodes % b else 0))):
                d_recvp[r] = None
    rc_ = group.phase_collective(PHASE_MODE[mode], d_sendp, d_recvp, rc, DT[dtype], OP[op], k, b)
    assert rc_ == 0, f"rc={rc_}"
    return [gu.from_dev(d, npdt, out_n) for d in d_recv]


def test_phases_match_reference_golden(gu, groups, golden_phases):
    """CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/reduce_scatter/:
    intra_reduce_scatter_radix_batch, inter_reduce_linear, intra_scatter_radix_batch): every golden case
    of the reference's own code bit-exact on the device (in place where the reference supports it;
    non-roots of the scatter pass no send buffer, as its self-test does)."""
    cases, _ = golden_phases
    bad = []
    for c in cases:
        n = c["n"]
        in_n, _ = po.phase_sizes(c["mode"], n, c["b"], c["count"])
        sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
        outs = _run_phase(gu, groups(n), c["mode"], sends, c["k"] or 2, c["b"], c["count"], c["dtype"], c["op"],
                          inplace=bool(c["inplace"]), null_unread=True)
        if hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest() != c["sha256"]:
            bad.append(c["id"])
    assert not bad, f"{len(bad)} device/reference mismatches, e.g. {bad[:5]}"


@pytest.mark.parametrize("mode,n,k,b", [("irs", 12, 2, 3), ("irs", 8, 4, 2), ("ilr", 12, 2, 2), ("isc", 9, 3, 9)])
def test_phases_large(gu, groups, mode, n, k, b):
    """MiB-sized chunks (the vector kernel paths, odd counts for the tails): bit-exact vs the oracle.
    irs 12/3: one stage plus a leftover stage and step-1 folds (b = 3 is not a power of 2)."""
    rc = (1 << 18) + 3
    in_n, _ = po.phase_sizes(mode, n, b, rc)
    sends = [po.fill(in_n, "f32", po.PAT_UNIFORM, 5, r) for r in range(n)]
    want = po.phase_collective(mode, sends, "f32", "sum", k, b, rc)
    got = _run_phase(gu, groups(n), mode, sends, k, b, rc, "f32", "sum")
    for r in range(n):
        np.testing.assert_array_equal(got[r].view(np.uint32), want[r].view(np.uint32))


def test_phases_reject_in_place_where_the_reference_does(gu, groups):
    """inter_reduce_linear and intra_scatter_radix_batch read sendbuf unconditionally (no MPI_IN_PLACE);
    here CHR_IN_PLACE is an error instead of a crash.  n % b != 0 is CHR_ERR_BATCH_NOT_DIVISOR."""
    n, b, rc = 4, 2, 8
    d = [gu.to_dev(np.zeros(64, dtype=np.float32)) for _ in range(n)]
    g = groups(n)
    for mode in (ca.MODE_INTER_REDUCE_LINEAR, ca.MODE_INTRA_SCATTER):
        assert g.phase_collective(mode, [ca.IN_PLACE] * n, d, rc, ca.FLOAT32, ca.SUM, 2, b) == ca.ERR_INVALID_ARG
    assert g.phase_collective(ca.MODE_INTRA_REDUCE_SCATTER, d, d, rc, ca.FLOAT32, ca.SUM, 2, 3) == ca.ERR_BATCH_NOT_DIVISOR
