"""Randomised parity on the GPU: every collective family (CHiArA's stand-alone phases included), geometry, schedule, pipeline depth, dtype,
op and in-place combination drawn from a seeded generator, each checked bit for bit against the
oracle (LocalGroup: the RCCL path's plans and kernels with device copies as messages).

The golden grids pin the reference's behaviour; this covers the combinations between them (odd
counts under every schedule and depth, batched trees with ragged pieces, the MPICH baselines with
non-default k, integer types through the flat plans).  A second run forces the streaming kernel
shapes (CHR_REDUCE_NT=1) with small XCD runs and small launch caps, so the one-wave nt kernels, the
XCD map and the launch/segment splitting run under the collectives at oracle sizes.  Each run is a
child process (the kernel tunables are read once per process)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [{here!r}, {oracle!r}, {pkg!r}]
import chiara_amd as ca
import gpu_util as gu
import pyoracle as po

DT = {{"f32": ca.FLOAT32, "f64": ca.FLOAT64, "i32": ca.INT32, "bf16": ca.BFLOAT16, "i8": ca.INT8, "u8": ca.UINT8,
      "i16": ca.INT16, "u16": ca.UINT16, "u32": ca.UINT32, "i64": ca.INT64, "u64": ca.UINT64}}
OP = {{"sum": ca.SUM, "prod": ca.PROD, "max": ca.MAX, "min": ca.MIN, "land": ca.LAND, "lor": ca.LOR,
      "lxor": ca.LXOR, "band": ca.BAND, "bor": ca.BOR, "bxor": ca.BXOR}}
PAIRS = [("f32", "sum"), ("f32", "sum"), ("f32", "max"), ("f32", "min"), ("f32", "prod"), ("bf16", "sum"),
         ("bf16", "max"), ("f64", "sum"), ("i32", "sum"), ("i32", "max"), ("i64", "bxor"), ("u8", "min"),
         ("i16", "land"), ("u32", "bor"), ("f32", "lor"), ("u64", "sum"), ("i8", "prod")]
SCHED = [ca.SCHEDULE_FLAT, ca.SCHEDULE_REFERENCE, ca.SCHEDULE_BALANCED, ca.SCHEDULE_EXACT, ca.SCHEDULE_FLAT_AG,
         ca.SCHEDULE_FLAT_SEQ, ca.SCHEDULE_FLAT_1SHOT]
MPICH = {{"ring": ca.MODE_MPICH_RING, "rd": ca.MODE_MPICH_RD, "rsag": ca.MODE_MPICH_RSAG, "rx": ca.MODE_MPICH_RECEXCH,
         "krsag": ca.MODE_MPICH_KRSAG, "rm": ca.MODE_MPICH_RMULT}}
MPICH_RS = {{"rs_radix": ca.MODE_MPICH_RS_RADIX, "rs_halving": ca.MODE_MPICH_RS_HALVING,
            "rs_doubling": ca.MODE_MPICH_RS_DOUBLING, "rs_pairwise": ca.MODE_MPICH_RS_PAIRWISE}}

if {userops}:  # user-defined ops (chr_op_create): the test launcher registered non-commutative and commutative
    import ctypes
    _lib = ctypes.CDLL({userop_so!r})
    _fn = ctypes.cast(_lib.chr_test_halfadd, ctypes.c_void_p).value
    OP["user_halfadd"] = ca.op_create(_fn, commute=False)
    OP["user_halfadd_c"] = ca.op_create(_fn, commute=True)
    PAIRS = [("f32", "user_halfadd"), ("f32", "user_halfadd"), ("f64", "user_halfadd"), ("i32", "user_halfadd"),
             ("f32", "user_halfadd_c"), ("i32", "user_halfadd_c")]
rng = np.random.default_rng({seed})
groups = {{}}
bad, done = [], 0
for case in range({ncases}):
    fam = rng.choice(["ar", "ar", "rs", "rs", "mpich", "mpich_rs", "phase"] if {userops} else
                     ["ar", "ar", "rs", "rs", "ag", "mpich", "mpich_rs", "phase"])
    n = int(rng.integers(1, 13))
    divs = [d for d in range(1, n + 1) if n % d == 0]
    b = int(rng.choice(divs))
    k = int(rng.integers(2, 10))
    dtype, op = PAIRS[int(rng.integers(len(PAIRS)))]
    if fam == "ag":
        op = "sum"
    algo = str(rng.choice(["irs", "ilr"] if {userops} else ["irs", "ilr", "isc"])) if fam == "phase" else None
    if algo == "isc":
        op = "sum"
    rc_ = int(rng.choice([1, 3, 17, 255, 256, 1000, 4097, 12345, 40000]))
    inplace = bool(rng.integers(2))
    pat = po.PAT_TIES if op in ("max", "min") and dtype in ("f32", "bf16", "f64") and rng.integers(2) else (
        po.PAT_SPARSE if dtype not in ("f32", "bf16", "f64") and rng.integers(2) else po.PAT_UNIFORM)
    seed = int(rng.integers(1 << 30))
    if n not in groups:
        groups[n] = ca.LocalGroup(n, 0)
    g = groups[n]
    g.set_schedule(int(rng.choice(SCHED)) if fam in ("ar", "rs") else ca.SCHEDULE_FLAT)
    g.set_slices(int(rng.integers(0, 6)))
    npdt = po.NP_DTYPES[dtype]
    es = np.dtype(npdt).itemsize
    tag = dict(case=case, fam=str(fam), n=n, b=b, k=k, dtype=dtype, op=op, rc=rc_, inplace=inplace)
    try:
        if fam in ("ar", "mpich"):
            count = rc_ * n
            sends = [po.fill(count, dtype, pat, seed, r) for r in range(n)]
            d_send = [gu.to_dev(s) for s in sends]
            d_recv, d_sendp = (d_send, [ca.IN_PLACE] * n) if inplace else ([gu.empty_dev(count * es) for _ in range(n)], d_send)
            if fam == "ar":
                rc = g.all_reduce_radix_batch(d_sendp, d_recv, count, DT[dtype], OP[op], k, b)
                want = po.allreduce_radix_batch(sends, k, b, dtype, op, inplace=inplace)
            else:
                algo = str(rng.choice(list(MPICH)))
                tag["algo"] = algo
                rc = g.allreduce_mpich(MPICH[algo], d_sendp, d_recv, count, DT[dtype], OP[op], k, 0)
                try:
                    want = po.mpich_allreduce(algo, sends, dtype, op, k=k, inplace=inplace)
                except ValueError as e:  # the reference's MPI_ERR_OP for a non-commutative op: refused alike
                    if not (len(e.args) > 1 and e.args[1] == po.ORC_ERR_OP and rc == ca.ERR_UNSUPPORTED):
                        raise
                    done += 1
                    continue
            outc = count
        elif fam in ("rs", "mpich_rs"):
            sends = [po.fill(rc_ * n, dtype, pat, seed, r) for r in range(n)]
            d_send = [gu.to_dev(s) for s in sends]
            d_recv, d_sendp = (d_send, [ca.IN_PLACE] * n) if inplace else ([gu.empty_dev(rc_ * es) for _ in range(n)], d_send)
            if fam == "rs":
                rc = g.reduce_scatter_radix_batch(d_sendp, d_recv, rc_, DT[dtype], OP[op], k, b)
                want = po.reduce_scatter_radix_batch(sends, k, b, dtype, op, inplace=inplace)
            else:
                algo = str(rng.choice(list(MPICH_RS)))
                tag["algo"] = algo
                rc = g.reduce_scatter_mpich(MPICH_RS[algo], d_sendp, d_recv, rc_, DT[dtype], OP[op], k)
                want = po.mpich_reduce_scatter(algo, sends, dtype, op, k=k, inplace=inplace)
            outc = rc_
        elif fam == "phase":  # CHiArA's stand-alone phases (in place: intra_reduce_scatter only)
            tag["algo"] = algo
            inplace = inplace and algo == "irs"
            tag["inplace"] = inplace
            in_n, outc = po.phase_sizes(algo, n, b, rc_)
            sends = [po.fill(in_n, dtype, pat, seed, r) for r in range(n)]
            if inplace:
                d_recv = [gu.to_dev(s_) for s_ in sends]
                d_sendp = [ca.IN_PLACE] * n
            else:
                d_recv = [gu.to_dev(np.zeros(max(outc, 1), dtype=npdt)) for _ in range(n)]
                d_sendp = [gu.to_dev(s_) for s_ in sends]
            mode = {{"irs": ca.MODE_INTRA_REDUCE_SCATTER, "ilr": ca.MODE_INTER_REDUCE_LINEAR,
                    "isc": ca.MODE_INTRA_SCATTER}}[algo]
            rc = g.phase_collective(mode, d_sendp, d_recv, rc_, DT[dtype], OP[op], k, b)
            want = po.phase_collective(algo, sends, dtype, op, k, b, rc_, inplace=inplace)
        else:
            sends = [po.fill(rc_, dtype, pat, seed, r) for r in range(n)]
            d_recv = [gu.empty_dev(rc_ * n * es) for _ in range(n)]
            if inplace:
                for r in range(n):
                    d_recv[r][r * rc_ * es:(r + 1) * rc_ * es].copy_(gu.to_dev(sends[r]))
                d_sendp = [ca.IN_PLACE] * n
            else:
                d_sendp = [gu.to_dev(s) for s in sends]
            rc = g.allgather_radix_batch(d_sendp, rc_, DT[dtype], d_recv, k, b)
            want = [np.concatenate(sends)] * n
            outc = rc_ * n
        gu.sync()
        if rc != 0:
            bad.append(dict(tag, rc=rc))
            continue
        for r in range(n):
            got = gu.from_dev(d_recv[r], npdt, outc)
            if got.tobytes() != np.ascontiguousarray(want[r][:outc]).tobytes():
                bad.append(dict(tag, rank=r))
                break
        done += 1
    except Exception as e:
        bad.append(dict(tag, error=str(e)[:200]))
for g in groups.values():
    g.destroy()
print(json.dumps({{"done": done, "bad": bad[:20], "nbad": len(bad)}}))
"""


def _run(seed, ncases, env_extra, userops=False):
    code = CHILD.format(here=HERE, oracle=os.path.join(REPO, "oracle"),
                        pkg=os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd"),
                        seed=seed, ncases=ncases, userops=userops,
                        userop_so=os.path.join(HERE, "userop", "libhalfadd_op.so"))
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_fuzz_collectives_default_policy():
    res = _run(20261016, 600, {})
    assert res["nbad"] == 0, res["bad"]
    assert res["done"] == 600


def test_fuzz_collectives_streaming_kernels_forced():
    res = _run(77, 400, {"CHR_REDUCE_NT": "1", "CHR_XCD_RUN_KIB": "4", "CHR_REDUCE_MAX_LAUNCH_VEC": "2048"})
    assert res["nbad"] == 0, res["bad"]
    assert res["done"] == 400



def test_fuzz_collectives_user_ops():
    """User-defined ops through every family but allgather (no op): the test launcher registered non-commutative
    and commutative, float / double / int32, every schedule and depth, the MPICH baselines' refusals of a
    non-commutative op included -- bit for bit against the oracle's restatement (ORC_USER_HALFADD)."""
    res = _run(606, 600, {}, userops=True)
    assert res["nbad"] == 0, res["bad"]
    assert res["done"] == 600
