"""The RCCL transport with several ranks on the single-GPU test box.

RCCL refuses two ranks on one device on the same host ("Duplicate GPU detected"), so
each rank process gets its own NCCL_HOSTID: RCCL then treats the ranks as separate hosts
and moves messages over its socket transport (loopback).  Same executor, same plans,
same kernels as the xGMI path on the 8-GPU node; only the wire differs.  Results must
be bit-exact vs the oracle."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    os.environ["NCCL_HOSTID"] = f"chiara-test-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    sys.path[:0] = [HERE, os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]
    import torch
    import torch.distributed as dist

    import chiara_amd as ca
    import pyoracle as po

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = ca.Comm.from_torch_distributed(device=0)
    dev = torch.device("cuda:0")
    try:
        for case in cases:
            (mode, k, b, count, dtype, host, slices), extra = case[:7], case[7:]
            comm.set_slices(slices)
            comm.set_schedule(extra[0] if extra else ca.SCHEDULE_FLAT)
            comm.set_overlap(extra[1] if len(extra) > 1 else True)
            inplace = len(extra) > 2 and extra[2]
            npdt = po.NP_DTYPES[dtype]
            cdt = {"f32": ca.FLOAT32, "bf16": ca.BFLOAT16, "i32": ca.INT32}[dtype]
            in_n = count * world if mode == "rs" else count
            out_n = count * world if mode == "ag" else count
            pat = po.PAT_TIES if mode == "rx" else 0  # recexch: operand-order sensitive data, MAX
            x = po.fill(in_n, dtype, pat, 4242, rank)
            if host:
                send, out = x, np.zeros(out_n, dtype=npdt)
            elif inplace:  # MPI_IN_PLACE: the input sits in the receive buffer
                out_t = torch.from_numpy(x.view(np.uint8).copy()).to(dev)
                send = ca.IN_PLACE
            else:
                send = torch.from_numpy(x.view(np.uint8).copy()).to(dev)
                out_t = torch.zeros(out_n * x.itemsize, dtype=torch.uint8, device=dev)
            dst = out if host else out_t
            allx = [po.fill(in_n, dtype, pat, 4242, r) for r in range(world)]
            if mode == "ag":
                rc = ca.allgather_radix_batch(send, count, cdt, dst, comm, k, b)
                ref = np.concatenate(allx)
            elif mode in ("ar", "rs"):
                fn = ca.all_reduce_radix_batch if mode == "ar" else ca.reduce_scatter_radix_batch
                rc = fn(send, dst, count, cdt, ca.SUM, comm, k, b)
                f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
                ref = f(allx, k, b, dtype, "sum")[rank]
            elif mode == "rx":
                rc = ca.MPICH_Allreduce_recursive_exchange(send, dst, count, cdt, ca.MAX, comm, k, b)
                ref = po.mpich_allreduce("rx", allx, dtype, "max", k=k)[rank]
            elif mode == "krsag":
                rc = ca.MPICH_Allreduce_k_reduce_scatter_allgather(send, dst, count, cdt, ca.SUM, comm, k, b)
                ref = po.mpich_allreduce("krsag", allx, dtype, "sum", k=k)[rank]
            elif mode == "rm":
                rc = ca.MPICH_Allreduce_recursive_multiplying(send, dst, count, cdt, ca.SUM, comm, k)
                ref = po.mpich_allreduce("rm", allx, dtype, "sum", k=k)[rank]
            else:
                fn = {"ring": ca.MPICH_Allreduce_ring, "rd": ca.MPICH_Allreduce_recursive_doubling,
                      "rsag": ca.MPICH_Allreduce_reduce_scatter_allgather}[mode]
                rc = fn(send, dst, count, cdt, ca.SUM, comm)
                ref = po.mpich_allreduce(mode, allx, dtype, "sum")[rank]
            if not host:
                out = out_t.cpu().numpy().view(npdt)[:out_n]
            ok = bool(np.array_equal(out.view(np.uint8), ref.view(np.uint8)))
            if extra and extra[0] == ca.SCHEDULE_AUTO and mode in ("ar", "rs"):
                # device calls keep a measured choice; host-staged ones run FLAT untuned
                tuned = comm.tuned_schedule(ca.MODE_ALLREDUCE if mode == "ar" else ca.MODE_REDUCE_SCATTER, count, cdt,
                                            k, b)
                ok = ok and ((tuned is None) == host)
                ok = ok and (tuned is None or tuned[0] in (ca.SCHEDULE_FLAT, ca.SCHEDULE_FLAT_SEQ, ca.SCHEDULE_FLAT_AG))
            q.put((rank, mode, k, b, rc, ok))
    finally:
        comm.destroy()
        dist.destroy_process_group()


def _run(world, cases, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "RCCL multi-rank test hung"
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get() for _ in range(world * len(cases))]
    bad = [r for r in res if r[4] != 0 or not r[5]]
    assert not bad, bad


def test_rccl_world2_reduce_scatter_and_allreduce():
    _run(2, [("rs", 2, 1, 1 << 16, "f32", False, 0), ("rs", 2, 2, 1 << 16, "f32", False, 3),
             ("ar", 2, 2, 1 << 16, "f32", False, 4), ("ar", 2, 1, 2 * 1001, "bf16", False, 0),
             ("ar", 2, 2, 1 << 14, "f32", True, 2)])


def test_rccl_world8_c4_c5_geometries():
    _run(8, [("ar", 4, 4, 8 * 4096, "f32", False, 0), ("ar", 4, 4, 8 * 4096, "bf16", False, 4),
             ("ar", 2, 2, 8 * 4096, "f32", False, 3), ("ar", 3, 4, 8 * 2048, "bf16", False, 2),
             ("ar", 4, 8, 8 * 1024, "f32", False, 0), ("rs", 4, 4, 4000, "f32", False, 3)], timeout=600)


def test_rccl_mpich_baselines_world5_and_8():
    """testing/main.cpp's baselines over RCCL, non-power-of-two (fold/unfold) and 8 ranks."""
    cases = [("ring", 0, 0, 100003, "f32", False, 0), ("rd", 0, 0, 4099, "f32", False, 0),
             ("rsag", 0, 0, 65537, "f32", True, 0), ("rx", 3, 0, 20000, "f32", False, 0),
             ("rx", 2, 1, 777, "bf16", False, 0), ("krsag", 2, 0, 30011, "f32", False, 0),
             ("rm", 2, 0, 4097, "f32", False, 0)]
    _run(5, cases)
    _run(8, cases[:1] + [("rx", 4, 0, 1 << 16, "f32", False, 0), ("rsag", 0, 0, 1 << 16, "bf16", False, 0),
                         ("krsag", 2, 1, 1 << 16, "f32", False, 0), ("rm", 3, 0, 12345, "bf16", False, 0)],
         timeout=600)


def test_rccl_allgather_world4_and_8():
    _run(4, [("ag", 2, 2, 1 << 16, "f32", False, 0), ("ag", 3, 4, 1001, "bf16", True, 0)])
    _run(8, [("ag", 4, 4, 1 << 18, "f32", False, 0), ("ag", 8, 2, 4097, "i32", False, 0)], timeout=600)


def test_rccl_schedules_and_overlap_world4():
    """The two-stream executor (overlap on/off) under all six schedules, allreduce and
    reduce-scatter, 4 ranks over RCCL: bit-exact vs the oracle."""
    cases = []
    for sched in (0, 1, 2, 3, 4, 5):
        for ov in (True, False):
            cases.append(("ar", 4, 4, 1 << 18, "f32", False, 4, sched, ov))
            cases.append(("rs", 2, 2, 1 << 15, "f32", False, 3, sched, ov))
    cases.append(("ar", 2, 4, 1 << 18, "bf16", False, 5, 2, True))  # multi-phase tree, flat
    _run(4, cases, timeout=600)


def test_rccl_auto_schedule_world4():
    """CHR_SCHEDULE_AUTO over RCCL: the first call per argument set times FLAT / FLAT_SEQ /
    FLAT_AG at several pipeline depths and every rank keeps the same one (a disagreement would
    hang); the result of the tuning call and of the cached later call is bit-exact vs the
    oracle, in place (tuned on copies: the caller's data is reduced once) and host-staged."""
    A = 6  # SCHEDULE_AUTO
    cases = [("ar", 4, 4, 1 << 18, "f32", False, 0, A, True), ("ar", 4, 4, 1 << 18, "f32", False, 0, A, True),
             ("ar", 2, 2, 1 << 16, "bf16", False, 0, A, True, True), ("ar", 2, 2, 1 << 16, "bf16", False, 0, A, True, True),
             ("rs", 2, 2, 1 << 15, "f32", False, 0, A, True), ("rs", 4, 4, 4000, "f32", False, 0, A, True, True),
             ("ar", 4, 4, 1 << 14, "f32", True, 0, A, True), ("ar", 2, 4, 8 * 1001, "bf16", False, 3, A, False)]
    _run(4, cases, timeout=600)


def test_rccl_exact_schedule_world8():
    """The reference's own messages end to end (bcast + left-over k-Bruck at C4; k-nomial
    scatter for reduce-scatter), 8 ranks over RCCL: bit-exact vs the oracle."""
    _run(8, [("ar", 4, 4, 1 << 18, "f32", False, 0, 3, True), ("ar", 2, 8, 8 * 1001, "bf16", False, 0, 3, True),
             ("ar", 2, 2, 1 << 16, "f32", True, 0, 3, False), ("rs", 4, 8, 1 << 14, "f32", False, 0, 3, True),
             ("rs", 2, 4, 999, "f32", False, 0, 3, True)], timeout=600)


def _phase_worker(rank, world, port, q):
    os.environ["NCCL_HOSTID"] = f"chiara-test-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    sys.path[:0] = [HERE, os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]
    import torch
    import torch.distributed as dist

    import chiara_amd as ca

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = ca.Comm.from_torch_distributed(device=0)
    try:
        count = 1 << 16
        send = torch.ones(count, dtype=torch.float32, device="cuda:0")
        recv = torch.zeros(count, dtype=torch.float32, device="cuda:0")
        out = {}
        for name, sch in (("flat", ca.SCHEDULE_FLAT), ("exact", ca.SCHEDULE_EXACT)):
            comm.set_schedule(sch)
            comm.profile(True)
            ca.check(ca.all_reduce_radix_batch(send, recv, count, ca.FLOAT32, ca.SUM, comm, 4, 4))
            comm.profile_read()
            out[name] = comm.profile_phases()
            comm.profile(False)
        q.put((rank, out, float(recv[7].item())))
    finally:
        comm.destroy()
        dist.destroy_process_group()


def test_rccl_profile_phases_world4():
    """chr_comm_profile_phases: per-phase transfer times named after the plan's phases."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_phase_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive and all(p.exitcode == 0 for p in procs)
    for _ in range(4):
        rank, out, v = q.get()
        assert v == 4.0
        assert set(out["flat"]) == {"gather", "fdist"}, out
        assert all(ms > 0 for ms in out["flat"].values())
        assert any(k.startswith("bruck") for k in out["exact"]) and "bcast" not in out["exact"], out


def _graph_worker(rank, world, port, q):
    os.environ["NCCL_HOSTID"] = f"chiara-test-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    sys.path[:0] = [HERE, os.path.join(REPO, "oracle"),
                    os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]
    import torch
    import torch.distributed as dist

    import chiara_amd as ca
    import pyoracle as po

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = ca.Comm.from_torch_distributed(device=0)
    dev = torch.device("cuda:0")
    comm.set_graphs(True)
    try:
        # (mode, k, b, count, dtype, slices, schedule, overlap): every call after the first replays the
        # graph captured for these buffers, so each round refills the same send buffer with new data
        for mode, k, b, count, dtype, slices, sched, ov in (
                ("ar", 4, 4, 1 << 16, "f32", 4, ca.SCHEDULE_FLAT, True),
                ("ar", 2, 4, 8 * 1001, "bf16", 2, ca.SCHEDULE_REFERENCE, True),
                ("rs", 2, 2, 1 << 14, "f32", 3, ca.SCHEDULE_FLAT_SEQ, False),
                ("ar", 4, 4, 1 << 15, "f32", 0, ca.SCHEDULE_AUTO, True)):
            comm.set_slices(slices)
            comm.set_schedule(sched)
            comm.set_overlap(ov)
            cdt = {"f32": ca.FLOAT32, "bf16": ca.BFLOAT16}[dtype]
            in_n = count * world if mode == "rs" else count
            es = 4 if dtype == "f32" else 2
            send = torch.empty(in_n * es, dtype=torch.uint8, device=dev)
            out_t = torch.empty(count * es, dtype=torch.uint8, device=dev)
            for rnd in range(3):
                seed = 777 + rnd
                send.copy_(torch.from_numpy(po.fill(in_n, dtype, 0, seed, rank).view(np.uint8).copy()))
                fn = ca.all_reduce_radix_batch if mode == "ar" else ca.reduce_scatter_radix_batch
                rc = fn(send, out_t, count, cdt, ca.SUM, comm, k, b)
                allx = [po.fill(in_n, dtype, 0, seed, r) for r in range(world)]
                f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
                ref = f(allx, k, b, dtype, "sum")[rank]
                out = out_t.cpu().numpy()
                q.put((rank, mode, k, b, rc, bool(np.array_equal(out, ref.view(np.uint8)))))
    finally:
        comm.set_graphs(False)
        comm.destroy()
        dist.destroy_process_group()


def test_rccl_graph_replay_world4():
    """chr_comm_set_graphs: the captured plan (RCCL groups + reductions on two streams) replays
    bit-exact vs the oracle on new data in the same buffers, for flat / reference / flat_seq
    (overlap off) / AUTO plans, allreduce and reduce-scatter."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "RCCL graph test hung"
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get() for _ in range(world * 4 * 3)]
    bad = [r for r in res if r[4] != 0 or not r[5]]
    assert not bad, bad
