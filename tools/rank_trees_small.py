#!/usr/bin/env python3
"""One GPU's own fused reductions of the N = 2 / N = 4 lines' allreduce (1 GiB fp32 per rank, flat schedule, b = N,
k = min(4, N)): rank 0's 2- or 4-leaf tree grids on its own send / recv / STAGE, with and without the receive
copies in front (bench.replay_rank_trees, the C4 / C5 rank-alone rows' method), at the in-collective cap when
CHR_WG_PER_CU_TREE=12 is set.  For A/Bs of tree-kernel policy on the shape the N = 2 / N = 4 lines run.
Measurement tooling only.

    python3 tools/rank_trees_small.py [--n 2] [--slices 4 8]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import chiara_amd as ca  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--slices", type=int, nargs="+", default=[4, 8])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = a.n
    k = min(4, n)
    for slices in a.slices:
        for recv_copies in (False, True):
            row = bench.replay_rank_trees(ca, torch, dev, ca.FLOAT32, 4, (1 << 30) // 4, n, k, n, slices, recv_copies,
                                          graph=False)
            print(json.dumps({"n": n, "slices": slices, "recv_copies": recv_copies,
                              "env": {k_: v for k_, v in os.environ.items() if k_.startswith("CHR_")}, **row}),
                  flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
