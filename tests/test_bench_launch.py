"""bench.py --gpus N starts its own rank processes (the reference's run target
starts its own ranks: testing/Makefile:83-87, `mpirun -np $(TOTAL_PROCS)`).  CPU-only: the launch
decision, the command, the too-many-ranks error, rank 0's line forwarded, the deadline."""
import json
import os
import subprocess
import sys

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(*argv):
    return bench.parse(list(argv))


def test_one_gpu_runs_in_process():
    assert bench.plan_launch(_args(), [], {}, 8) is None
    assert bench.plan_launch(_args("--gpus", "1"), ["--gpus", "1"], {}, 8) is None


def test_external_launcher_rank_runs_in_process():
    argv = ["--gpus", "8"]
    assert bench.plan_launch(_args(*argv), argv, {"WORLD_SIZE": "8", "RANK": "3"}, 8) is None


def test_gpus_n_spawns_torchrun_child():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.plan_launch(_args(*argv), argv, {}, 8, port=29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(REPO, "bench.py") and cmd[-len(argv):] == argv


def test_too_many_ranks_is_an_error():
    argv = ["--gpus", "8"]
    with pytest.raises(ValueError, match="only 1 GPU"):
        bench.plan_launch(_args(*argv), argv, {}, 1)
    with pytest.raises(ValueError):
        bench.plan_launch(_args(*argv), argv, {}, 0)
    # a rehearsal with ranks sharing one GPU is allowed explicitly
    assert bench.plan_launch(_args(*argv), argv, {"CHR_BENCH_VIRTUAL_HOSTS": "1"}, 1)


def test_cli_too_many_ranks_exits_nonzero_without_a_line():
    """No GPU in this container: --gpus 2 must fail loudly, not print the one-GPU line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "CHR_BENCH_VIRTUAL_HOSTS")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 2 and r.stdout.strip() == "" and "GPU(s) visible" in r.stderr


def test_launcher_forwards_rank0_line_and_exit_status(capsys):
    line = {"metric": bench.METRIC, "value": 1.0, "n_gpus": 2}
    child = ("import json,sys; print('banner noise'); print(json.dumps(%r)); sys.stdout.flush(); "
             "sys.exit(0)" % line)
    rc = bench.run_launcher([sys.executable, "-c", child])
    out = capsys.readouterr()
    assert rc == 0 and json.loads(out.out.strip()) == line and "banner noise" in out.err
    rc = bench.run_launcher([sys.executable, "-c", "import sys; sys.exit(3)"])
    assert rc == 3 and capsys.readouterr().out == ""


def test_launcher_passes_the_launch_time():
    rc = bench.run_launcher([sys.executable, "-c",
                             "import os,json,time; t=float(os.environ['CHR_BENCH_T0']); "
                             "assert abs(time.time()-t) < 60; print(json.dumps({'metric': 'm', 't0': t}))"])
    assert rc == 0


def test_deadline_agreed_over_ranks(monkeypatch):
    """Rank 0's decision is broadcast (gloo, one process here): past the deadline -> skipped entries."""
    import torch.distributed as dist

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(bench.free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        import time

        d = bench.Deadline(dist, {"CHR_BENCH_T0": repr(time.time()), "CHR_BENCH_DEADLINE_S": "3600"})
        assert not d.passed()
        d = bench.Deadline(dist, {"CHR_BENCH_T0": repr(time.time() - 10), "CHR_BENCH_DEADLINE_S": "5"})
        assert d.passed()
    finally:
        dist.destroy_process_group()


def _deadline_worker(rank, world, port, q):
    import time

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0 is past its deadline, rank 1 is not: both must take rank 0's decision
        t0 = time.time() - (100 if rank == 0 else 0)
        d = bench.Deadline(dist, {"CHR_BENCH_T0": repr(t0), "CHR_BENCH_DEADLINE_S": "50"})
        q.put((rank, d.passed()))
    finally:
        dist.destroy_process_group()


def test_deadline_decision_is_rank0s_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    procs = [ctx.Process(target=_deadline_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_launcher_kills_a_rank_group_past_its_limit(monkeypatch):
    """A rank group still running at deadline + grace is killed as a process group (exit 124), so a
    hung N>1 line cannot hold the node."""
    import time

    monkeypatch.setattr(bench, "KILL_GRACE_S", 1.0)
    monkeypatch.setenv("CHR_BENCH_DEADLINE_S", "0.5")
    t0 = time.time()
    rc = bench.run_launcher([sys.executable, "-c", "import time; time.sleep(60)"])
    assert rc == 124 and time.time() - t0 < 30
