"""bench.result_check on CPU (gloo, world 2): the N>1 line's own output check passes on a correct allreduce
and catches the two ways a transport can go wrong -- ranks that disagree, and bytes that are stale or
misplaced -- without the oracle (bench.py's metric leg may not touch it)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
COUNT = 3000  # not a multiple of the window: the last window is ragged


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(torch, world, es):
    g = torch.Generator().manual_seed(1234)
    tdt = torch.float32 if es == 4 else torch.bfloat16
    return [(torch.rand(COUNT, generator=g) * 2 - 1).to(tdt) for _ in range(world)]


def _worker(rank, world, port, es, fault, q):
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        xs = _inputs(torch, world, es)
        # an allreduce's result: the inputs summed left to right in the working precision, per step rounded
        acc = xs[0].clone()
        for x in xs[1:]:
            acc = (acc.float() + x.float()).to(acc.dtype)
        if fault == "one_rank_differs" and rank == 1:
            acc[17] = torch.nextafter(acc[17].float(), torch.tensor(9.0)).to(acc.dtype)
        if fault == "stale_block":  # every rank got a stale copy of one block: one rank's input, not the sum
            acc[1000:1100] = xs[0][1000:1100]
        recv = acc.view(torch.uint8).clone()

        def fill_rank(r, buf):
            buf.view(xs[r].dtype)[:COUNT].copy_(xs[r])

        res = bench.result_check(torch, dist, recv, COUNT, es, world, fill_rank, window=1024)
        send = torch.zeros(COUNT * es, dtype=torch.uint8)
        out = torch.zeros(COUNT * es, dtype=torch.uint8)

        def run():  # an allreduce of the known-answer inputs (gloo sums integer-valued floats exactly)
            x = send.view(xs[0].dtype).float()
            dist.all_reduce(x)
            if fault == "exact_off_by_one" and rank == 1:
                x[2999] += 1
            out.view(xs[0].dtype).copy_(x.to(xs[0].dtype))

        res.update(bench.exact_check(torch, dist, send, out, COUNT, es, rank, run, world, window=1024))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _run(es, fault):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, es, fault, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("es", [4, 2])
def test_correct_allreduce_passes(es):
    out = _run(es, None)
    for r in (0, 1):
        c = out[r]
        assert c["ranks_bit_identical"] and c["within_tolerance"] and c["violations"] == 0, c
        assert c["elements_checked_per_rank"] == COUNT and c["max_err_over_bound"] <= 1.0
    assert out[0]["checksum_rank0"] == out[1]["checksum_rank0"]


@pytest.mark.parametrize("es", [4, 2])
def test_exact_known_answer(es):
    """The known-answer call: integer-valued inputs, every element equal to the sum -- passes on a correct allreduce
    (f32 and bf16: the partial sums stay exact), fails on one wrong element of one rank."""
    for r, c in _run(es, None).items():
        assert c["exact_known_answer"] and c["exact_violations"] == 0, c
    c = _run(es, "exact_off_by_one")[0]
    assert c["exact_known_answer"] is False and c["exact_violations"] == 1


def test_one_rank_differing_is_caught():
    c = _run(4, "one_rank_differs")[0]
    assert c["ranks_bit_identical"] is False
    assert c["within_tolerance"]  # one ulp is inside the tolerance: only the checksums see it


def test_stale_block_is_caught():
    c = _run(4, "stale_block")[0]
    assert c["ranks_bit_identical"]  # every rank has the same wrong bytes
    assert c["within_tolerance"] is False and c["violations"] >= 2 * 90


def test_line_problems_flags_a_failed_check():
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    from test_bench_line import _nn_line

    line = _nn_line()
    assert bench.line_problems(line) == []
    line["result_check"]["exact_known_answer"] = False
    assert any("exact known answer failed" in p for p in bench.line_problems(line))
    line["result_check"]["exact_known_answer"] = True
    line["result_check"]["within_tolerance"] = False
    assert any("result_check failed" in p for p in bench.line_problems(line))
    line.pop("result_check")
    assert any("result_check missing" in p for p in bench.line_problems(line))


def test_line_problems_flags_a_failed_n1_check():
    """The N = 1 line's own check (bench.bucket_result_check: one more launch, every element == torch's fp32 add):
    absent on older lines is fine, a failed one is a problem."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    from test_bench_line import _n1_line

    line = _n1_line()
    assert bench.line_problems(line) == []
    line["result_check"] = {"bit_exact_vs_torch_add": True, "mismatches": 0, "elements": 16}
    assert bench.line_problems(line) == []
    line["result_check"] = {"bit_exact_vs_torch_add": False, "mismatches": 3, "elements": 16}
    assert any("result_check failed" in p for p in bench.line_problems(line))
