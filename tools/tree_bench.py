#!/usr/bin/env python3
"""Fused expression tree vs one launch per fold, at the flat schedule's C4 evaluation shape.

C4 (n=8, k=4, b=4): each rank evaluates, per chunk, ((l0 l1 l2 l3) (l4 l5 l6 l7)) -- two
recexch folds of 4 (all_reduce_radix_batch.cpp:364) and the lane fold (:529).  Per-fold
launches move 13 x piece bytes (two m=3 folds + one m=1 fold); the tree kernel 9 x.
Prints one JSON line: time per evaluation and algorithmic GB/s of each form."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402

COMB, SWAPS = [0, 1, 1, 1, 0, 1, 1, 2], [0] * 7


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    out = {}
    for dname, cdt, tdt, es in (("f32", ca.FLOAT32, torch.float32, 4), ("bf16", ca.BFLOAT16, torch.bfloat16, 2)):
        out[dname] = run(dev, s, cdt, tdt, es)
    batched = {dname: run_batched(dev, s, cdt, tdt, es)
               for dname, cdt, tdt, es in (("f32", ca.FLOAT32, torch.float32, 4), ("bf16", ca.BFLOAT16, torch.bfloat16, 2))}
    print(json.dumps({"tree_vs_folds_c4": out, "slice_batched_c4": batched}))


def run_batched(dev, s, cdt, tdt, es):
    """The flat schedule at C4 evaluates, per pipeline slice, the trees of the 2 chunks (8 leaves x
    piece each).  Two launches (one per chunk) vs one batched launch (chr_reduce_tree_batch), with
    the leaves cold (cycled over a > 2 GiB working set) and warm (7 of 8 leaves just written by a
    device copy, as RCCL's receives leave them; only the tree launches are timed)."""
    out = {}
    for mib in (8, 16, 32):
        n = (mib << 20) // es
        sets = max(2, min(8, (2048 << 20) // (2 * 9 * es * n)))
        bufs = []
        for si in range(sets):
            trees = []
            for t in range(2):
                leaves = [torch.empty(n, dtype=tdt, device=dev) for _ in range(8)]
                for j, x in enumerate(leaves):
                    ca.fill(x, n, cdt, 0, 7, 16 * si + 8 * t + j, stream=s)
                trees.append((leaves, torch.empty(n, dtype=tdt, device=dev)))
            bufs.append(trees)
        src = torch.empty(n, dtype=tdt, device=dev)
        ca.fill(src, n, cdt, 0, 9, 0, stream=s)
        reps = 32

        def separate(i):
            rc = 0
            for lv, o in bufs[i % sets]:
                rc |= ca.reduce_tree(o, lv, COMB, SWAPS, n, cdt, ca.SUM, s)
            return rc

        def batched(i):
            tr = bufs[i % sets]
            return ca.reduce_tree_batch([o for _, o in tr], [lv for lv, _ in tr], [COMB, COMB], [SWAPS, SWAPS], n, cdt,
                                        ca.SUM, s)

        res = {}
        for name, fn in (("separate", separate), ("batched", batched)):
            for warm in (False, True):
                for i in range(3):
                    assert fn(i) == 0
                torch.cuda.synchronize()
                total = 0.0
                evs = []
                for i in range(reps):
                    if warm:
                        for lv, _ in bufs[i % sets]:
                            for x in lv[1:]:
                                x.copy_(src)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    fn(i)
                    e1.record(s)
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                total = sum(a.elapsed_time(b) for a, b in evs)
                us = total / reps * 1e3
                nbytes = 2 * 9 * es * n
                res[f"{name}_{'warm' if warm else 'cold'}"] = {
                    "us": round(us, 2), "GBps": round(nbytes / (us * 1e-6) / 1e9, 1),
                    "frac": round(nbytes / (us * 1e-6) / 8e12, 4)}
        tr = bufs[0]
        separate(0)
        ref = [o.clone() for _, o in tr]
        batched(0)
        torch.cuda.synchronize()
        res["bit_identical"] = all(bool(torch.equal(a.view(torch.int16), o.view(torch.int16)))
                                   for a, (_, o) in zip(ref, tr))
        out[f"piece_{mib}MiB"] = res
        del bufs
        torch.cuda.empty_cache()
    return out


def run(dev, s, cdt, tdt, es):
    out = {}
    for mib in (8, 64, 128):
        n = (mib << 20) // es
        sets = max(1, min(8, (2048 << 20) // (11 * es * n)))
        bufs = []
        for si in range(sets):
            leaves = [torch.empty(n, dtype=tdt, device=dev) for _ in range(8)]
            for j, t in enumerate(leaves):
                ca.fill(t, n, cdt, 0, 7, 8 * si + j, stream=s)
            bufs.append((leaves, torch.empty(n, dtype=tdt, device=dev),
                         torch.empty(n, dtype=tdt, device=dev), torch.empty(n, dtype=tdt, device=dev)))
        reps = 40

        def tree(i):
            lv, o, _, _ = bufs[i % sets]
            return ca.reduce_tree(o, lv, COMB, SWAPS, n, cdt, ca.SUM, s)

        def folds(i):
            lv, o, t0, t1 = bufs[i % sets]
            rc = ca.reduce_multi(t0, lv[0], lv[1:4], n, cdt, ca.SUM, s)
            rc |= ca.reduce_multi(t1, lv[4], lv[5:8], n, cdt, ca.SUM, s)
            return rc | ca.reduce_multi(o, t0, [t1], n, cdt, ca.SUM, s)

        res = {}
        for name, fn, nbytes in (("tree", tree, 9 * es * n), ("folds", folds, 13 * es * n)):
            for i in range(3):
                assert fn(i) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for i in range(reps):
                fn(i)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res[name] = {"us": round(ms * 1e3, 2), "alg_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                         "tree_bytes_GBps": round(9 * es * n / (ms * 1e-3) / 1e9, 1)}
        lv, o, t0, t1 = bufs[0]
        tree(0)
        a = o.clone()
        folds(0)
        torch.cuda.synchronize()
        res["bit_identical"] = bool(torch.equal(a.view(torch.int16), o.view(torch.int16)))
        res["speedup"] = round(res["folds"]["us"] / res["tree"]["us"], 3)
        out[f"piece_{mib}MiB"] = res
        del bufs
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
