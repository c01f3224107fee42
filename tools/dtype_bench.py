"""Bucket-kernel rates for the types and ops the C2 bench does not cover (8-bit and friends), HBM-cold.

chr_reduce_multi(acc, ins[m]) at `--mib` MiB per operand over a rotation of operand sets (> the 256 MiB Infinity
Cache), gated back-to-back launches timed with HIP events on one stream; fraction of 8 TB/s on the algorithmic
(m + 2) x bytes.  One JSON line per (dtype, op, m).  Used for the round-5 SWAR 8-bit A/B (tools/ab_old's library
against the in-tree one, swapped in place on the box: profiles/r05/dtype_ab/).

    python3 tools/dtype_bench.py [--mib 64] [--reps 30] [--label new]
"""
import argparse
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "configurable-hierarchical-allreduce-algorithms_amd"))
import chiara_amd as ca  # noqa: E402

CASES = [("u8", ca.UINT8, 1), ("i8", ca.INT8, 1), ("i16", ca.INT16, 2), ("i32", ca.INT32, 4)]
OPS = [("sum", ca.SUM), ("prod", ca.PROD), ("max", ca.MAX), ("min", ca.MIN), ("land", ca.LAND)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    nb = a.mib << 20
    for m in (1, 3):
        nsets = max(2, (2 << 30) // ((m + 1) * nb))  # > 2 GiB of distinct operands per rotation
        sets = [[torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(m + 1)] for _ in range(nsets)]
        for st in sets:
            for t in st:
                t.random_(0, 256)
        for dname, dt, es in CASES:
            n = nb // es
            for oname, op in OPS:
                def launch(i):
                    st = sets[i % nsets]
                    rc = ca.reduce_multi(st[0].data_ptr(), st[0].data_ptr(), [t.data_ptr() for t in st[1:]], n, dt,
                                         op, s)
                    assert rc == 0, rc
                for i in range(3):
                    launch(i)
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for i in range(a.reps):
                    launch(i)
                e1.record(s)
                torch.cuda.synchronize(dev)
                us = e0.elapsed_time(e1) * 1e3 / a.reps
                gbs = (m + 2) * nb / us / 1e3
                print(json.dumps({"label": a.label, "dtype": dname, "op": oname, "m": m, "mib": a.mib,
                                  "us": round(us, 2), "GBps": round(gbs, 1), "frac": round(gbs / 8000, 4)}),
                      flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
