#!/usr/bin/env python3
"""The 2-leaf tree against the C2 bucket kernel at identical traffic (2 reads + 1 write of 64 MiB per launch, f32
SUM), VERDICT r5 next-3: where does the 2-leaf tree's gap come from?  Variants, each timed as K gated back-to-back
launches (HIP events on the launch stream, like bench.py), over a rotation of distinct buffer sets:

  vec_inplace   chr_reduce_multi(out = acc, acc, [in])          -- C2 itself
  vec_oop       chr_reduce_multi(out, acc, [in]), out separate   -- the bucket kernel out of place
  tree_oop      chr_reduce_tree(out, [l0, l1])                   -- the N = 2 line's tree (out = the recv buffer)
  tree_inplace  chr_reduce_tree(out = l0, [l0, l1])

at a 2 GiB and a 4 GiB rotation (the bench rotates 2 GiB; tools/tree_pmc.py's 2-leaf sets total 4 GiB, past the
~2.5 GiB translation cliff of DESIGN §4.1).  Prints one JSON line per (variant, rotation, round).

    python3 tools/leaf2_ab.py [--rounds 2] [--launches 40]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

MIB = 1 << 20
PIECE = 64 * MIB


def timed(s, launches, fn):
    torch.cuda.synchronize()
    torch.cuda._sleep(2_000_000)  # gate: the host enqueues events and launches while the stream waits
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(launches):
        fn(i)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / launches  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--launches", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    n = PIECE // 4
    by = 3 * PIECE
    for rot_gib in (2, 4):
        nsets = rot_gib * 1024 // (3 * 64)  # three distinct 64 MiB buffers per set
        bufs = [[torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)] for _ in range(nsets)]
        for si, b in enumerate(bufs):
            for j, t in enumerate(b):
                ca.check(ca.fill(t, n, ca.FLOAT32, 0, 3, 3 * si + j, stream=s))
        variants = {
            "vec_inplace": lambda i: ca.check(ca.reduce_multi(bufs[i % nsets][0], bufs[i % nsets][0],
                                                              [bufs[i % nsets][1]], n, ca.FLOAT32, ca.SUM, s)),
            "vec_oop": lambda i: ca.check(ca.reduce_multi(bufs[i % nsets][2], bufs[i % nsets][0],
                                                          [bufs[i % nsets][1]], n, ca.FLOAT32, ca.SUM, s)),
            "tree_oop": lambda i: ca.check(ca.reduce_tree(bufs[i % nsets][2], bufs[i % nsets][:2], [0, 1], [0], n,
                                                          ca.FLOAT32, ca.SUM, s)),
            "tree_inplace": lambda i: ca.check(ca.reduce_tree(bufs[i % nsets][0], bufs[i % nsets][:2], [0, 1], [0],
                                                              n, ca.FLOAT32, ca.SUM, s)),
        }
        for name, fn in variants.items():  # warm every set once (page tables, first touch)
            timed(s, nsets, fn)
        for r in range(a.rounds):
            order = list(variants) if r % 2 == 0 else list(reversed(variants))
            for name in order:
                us = timed(s, a.launches, variants[name])
                print(json.dumps({"variant": name, "rotation_gib": round(nsets * 3 * 64 / 1024, 2), "round": r,
                                  "us_per_launch": round(us, 2),
                                  "frac": round(by / (us * 1e-6) / 8e12, 4)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
