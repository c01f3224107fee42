#!/usr/bin/env python3
"""Launches only the fused tree kernel at C4's shape (f32, 8 leaves, 64 MiB pieces, 8 rotating
leaf sets = 4.5 GiB, HBM-cold) for rocprofv3 --pmc passes: HBM bytes per launch vs the
algorithmic 9 x 64 MiB (tools/pmc_summary.py ... k_reduce_tree).  `--leaves 4|2`: the 4- / 2-leaf trees
instead ((L + 1) x 64 MiB; a streaming 2-leaf tree runs on the bucket kernel, reduce_tree.hip).  `--vec M --mib P`: the N = 2 / N = 4 lines' reductions instead -- one fold of M
incoming pieces of P MiB into a separate output (chr_reduce_multi(out, acc, ins), k_reduce_vec out of place,
(M + 2) x P MiB), over rotating sets of at least 4.5 GiB.

    python3 tools/tree_pmc.py [launches] [--leaves L | --vec M --mib P]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

COMBS = {8: [0, 1, 1, 1, 0, 1, 1, 2], 4: [0, 1, 0, 2], 2: [0, 1]}  # the flat schedule's programs at b = 8 / 4 / 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("launches", type=int, nargs="?", default=40)
    ap.add_argument("--leaves", type=int, default=8, choices=sorted(COMBS))
    ap.add_argument("--vec", type=int, default=0)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--rot-gib", type=float, default=4.5,
                    help="distinct operand bytes per rotation (4.5: past the translation cliff, the PMC runs' "
                         "setting; 1.9: C2's side of it, DESIGN §4.1)")
    a = ap.parse_args()
    if a.vec:
        return vec_oop(a)
    nl, comb = a.leaves, COMBS[a.leaves]
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    n = (64 << 20) // 4
    sets = []
    nsets = max(8, 64 // (nl + 1)) if a.rot_gib >= 4.5 else max(1, int(a.rot_gib * 16 // (nl + 1)))
    for si in range(nsets):  # >= 4.5 GiB of distinct operands per rotation by default
        leaves = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(nl)]
        for j, t in enumerate(leaves):
            ca.check(ca.fill(t, n, ca.FLOAT32, 0, 3, 8 * si + j, stream=s))
        sets.append((leaves, torch.empty(n, dtype=torch.float32, device=dev)))
    for i in range(a.launches):
        lv, o = sets[i % len(sets)]
        ca.check(ca.reduce_tree(o, lv, comb, [0] * (nl - 1), n, ca.FLOAT32, ca.SUM, s))
    torch.cuda.synchronize()
    print("tree launches done")


def vec_oop(a):
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    m, n = a.vec, (a.mib << 20) // 4
    sets = []
    nsets = (max(2, -(-(9 * 8 * 64) // ((m + 2) * a.mib))) if a.rot_gib >= 4.5
             else max(1, int(a.rot_gib * 1024 // ((m + 2) * a.mib))))
    for si in range(nsets):  # >= 4.5 GiB of distinct operands per rotation by default
        bufs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(m + 2)]
        for j, t in enumerate(bufs):
            ca.check(ca.fill(t, n, ca.FLOAT32, 0, 3, 16 * si + j, stream=s))
        sets.append(bufs)
    for i in range(a.launches):
        b = sets[i % len(sets)]
        ca.check(ca.reduce_multi(b[m + 1], b[0], b[1:m + 1], n, ca.FLOAT32, ca.SUM, s))
    torch.cuda.synchronize()
    print("reduce launches done")


if __name__ == "__main__":
    main()
