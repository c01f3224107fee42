#!/usr/bin/env python3
"""One GPU's own C4 / C5 tree grids by kernel duration: rocprofv3 --kernel-trace of `bench.py --rank-trees`
(tools/gpu.sh ranktrees), against the algorithmic bytes per grid of the same rows in rank_trees.json.
bench_rank_trees runs its rows in a fixed order and each row launches a fixed number of tree grids (2 warm
calls, `reps` spanned calls, `reps` calls with event pairs: 12 calls of launches_per_call grids), so the
trace's tree dispatches, in start order, split into the rows exactly; the split is checked against the
kernel symbol (f32 / bf16) of every dispatch.  Prints one JSON object.

usage: tools/rank_trees_summary.py <rank_trees.json> <dir with *kernel_trace.csv> [calls per row, default 12]"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    rows = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["rank_trees"]["rows"]
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    trace = sorted(glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True))[0]
    disp = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(trace)) if "k_reduce_tree<" in r["Kernel_Name"] or "k_reduce_tree_staged<" in r["Kernel_Name"]))
    need = sum(calls * v["launches_per_call"] for v in rows.values())
    if len(disp) != need:
        raise SystemExit(f"{len(disp)} tree dispatches in the trace, the rows account for {need}")
    out, i = {}, 0
    for key, v in rows.items():
        n = calls * v["launches_per_call"]
        mine = disp[i:i + n]
        i += n
        dt = "<3," if "bf16" in key else "<0,"
        if not all(("k_reduce_tree" + dt) in name.replace(" ", "") or ("k_reduce_tree_staged" + dt) in name.replace(" ", "")
                   for _, _, name in mine):
            raise SystemExit(f"row {key}: dispatches of another kernel in its slice of the trace")
        durs = [(e - s) / 1e3 for s, e, _ in mine[2 * v["launches_per_call"]:]]  # past the 2 warm-up calls
        by = v["algorithmic_bytes_per_call"] / v["launches_per_call"]
        avg, med = statistics.mean(durs), statistics.median(durs)
        out[key] = {"dispatches": len(durs), "avg_us": round(avg, 2), "median_us": round(med, 2),
                    "algorithmic_bytes_per_grid": int(by), "frac_avg": round(by / (avg * 1e-6) / 8e12, 4),
                    "frac_median": round(by / (med * 1e-6) / 8e12, 4),
                    "span_frac": v["frac"], "event_pairs_frac": v["event_pairs_frac"]}
    print(json.dumps({"rank_trees_rocprof": out, "trace": os.path.relpath(trace)}, indent=1))


if __name__ == "__main__":
    main()
