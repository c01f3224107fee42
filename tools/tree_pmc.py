#!/usr/bin/env python3
"""Launches only the fused tree kernel at C4's shape (f32, 8 leaves, 64 MiB pieces, 8 rotating
leaf sets = 4.5 GiB, HBM-cold) for rocprofv3 --pmc passes: HBM bytes per launch vs the
algorithmic 9 x 64 MiB (tools/pmc_summary.py ... k_reduce_tree)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

COMB = [0, 1, 1, 1, 0, 1, 1, 2]


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    n = (64 << 20) // 4
    sets = []
    for si in range(8):
        leaves = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(8)]
        for j, t in enumerate(leaves):
            ca.check(ca.fill(t, n, ca.FLOAT32, 0, 3, 8 * si + j, stream=s))
        sets.append((leaves, torch.empty(n, dtype=torch.float32, device=dev)))
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
        lv, o = sets[i % len(sets)]
        ca.check(ca.reduce_tree(o, lv, COMB, [0] * 7, n, ca.FLOAT32, ca.SUM, s))
    torch.cuda.synchronize()
    print("tree launches done")


if __name__ == "__main__":
    main()
