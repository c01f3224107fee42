#!/usr/bin/env python3
"""The N = 4 / N = 2 lines' 4- and 2-leaf trees alone, HBM-cold: one launch of 64 MiB pieces, and a slice grid of two
trees of 16 MiB pieces; gated back-to-back launches timed with HIP events on one stream, fraction of 8 TB/s on the
algorithmic (L + 1) x bytes.  The shape knobs come from the environment (CHR_XCD_RUN_KIB, CHR_WG_PER_CU_TREE), so
tools/gpu_small_tree_ab.sh runs this once per variant, alternating.  One JSON line per (leaves, shape).

    python3 tools/small_tree_ab.py --label NAME
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

COMBS = {4: [0, 1, 0, 2], 2: [0, 1]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    for nl in (4, 2):
        for piece_mib, ntrees in ((64, 1), (16, 2)):
            n = (piece_mib << 20) // 4
            per_set = ntrees * (nl + 1) * (piece_mib << 20)
            nsets = max(2, (3 << 30) // per_set)  # > 3 GiB of distinct operands per rotation
            sets = []
            for si in range(nsets):
                lv = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(ntrees * nl)]
                for j, t in enumerate(lv):
                    ca.check(ca.fill(t, n, ca.FLOAT32, 0, 3, 16 * si + j, stream=s))
                outs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(ntrees)]
                sets.append((lv, outs))

            def launch(i):
                lv, outs = sets[i % nsets]
                if ntrees == 1:
                    ca.check(ca.reduce_tree(outs[0], lv, COMBS[nl], [0] * (nl - 1), n, ca.FLOAT32, ca.SUM, s))
                else:
                    ca.check(ca.reduce_tree_batch(outs, [lv[t * nl:(t + 1) * nl] for t in range(ntrees)],
                                                  [COMBS[nl]] * ntrees, None, n, ca.FLOAT32, ca.SUM, s))
            for i in range(4):
                launch(i)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(a.reps):
                launch(i)
            e1.record(s)
            torch.cuda.synchronize(dev)
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            frac = per_set / us / 1e3 / 8000
            print(json.dumps({"label": a.label, "leaves": nl, "piece_mib": piece_mib, "trees": ntrees,
                              "us": round(us, 2), "frac": round(frac, 4),
                              "env": {k: os.environ.get(k) for k in ("CHR_XCD_RUN_KIB", "CHR_WG_PER_CU_TREE")}}),
                  flush=True)
            del sets
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
