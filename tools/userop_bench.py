"""User-defined op (chr_op_create) against the predefined SUM on the same shapes: the fold (MPI_Reduce_local, 64 MiB
buckets, m = 1 and 3, HBM-cold rotation) and an 8-virtual-rank C4-shaped allreduce (k = 4, b = 4, the flat
schedule's 8-leaf trees, evaluated for a user op as chained folds, user_ops.cpp user_tree).  One JSON line.
Measurement tool; the user op is tests/userop/halfadd_op.hip (one mul + one add per element, like SUM's one add)."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd"))
import chiara_amd as ca  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    lib = ctypes.CDLL(os.environ.get("CHR_USEROP_SO", os.path.join(REPO, "tests", "userop", "libhalfadd_op.so")))
    out_tag = os.environ.get("CHR_USEROP_SO", "")
    half = ca.op_create(ctypes.cast(lib.chr_test_halfadd, ctypes.c_void_p).value)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    out = {"tool": "tools/userop_bench.py", "lib": os.path.basename(out_tag) or "libhalfadd_op.so"}
    n = 16 << 20  # 64 MiB fp32
    for m in (1, 3):
        sets = max(1, (2 << 30) // ((m + 1) * 4 * n))
        bufs = [[torch.rand(n, device=dev) for _ in range(m + 1)] for _ in range(sets)]
        for name, op in (("sum", ca.SUM), ("user", half)):
            def go(i, op=op):
                s = bufs[i % sets]
                ca.check(ca.reduce_multi(s[0], s[0], s[1:], n, ca.FLOAT32, op, stream))
            ms = timed(go, 60)
            out[f"fold_m{m}_{name}_GBps"] = round((m + 2) * 4 * n / (ms * 1e-3) / 1e9, 1)
        del bufs
    nr, cnt = 8, 8 * (4 << 20)  # 128 MiB per rank
    g = ca.LocalGroup(nr, 0)
    sends = [torch.rand(cnt, device=dev) for _ in range(nr)]
    recvs = [torch.empty(cnt, device=dev) for _ in range(nr)]
    import time

    for name, op in (("sum", ca.SUM), ("user", half)):
        for _ in range(2):
            ca.check(g.all_reduce_radix_batch(sends, recvs, cnt, ca.FLOAT32, op, 4, 4))
        torch.cuda.synchronize()  # device-wide: the group's own stream included
        t0 = time.perf_counter()
        for _ in range(5):
            ca.check(g.all_reduce_radix_batch(sends, recvs, cnt, ca.FLOAT32, op, 4, 4))
        torch.cuda.synchronize()
        out[f"localgroup8_k4b4_128MiB_{name}_ms"] = round((time.perf_counter() - t0) / 5 * 1e3, 3)
    g.destroy()
    ca.op_free(half)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
