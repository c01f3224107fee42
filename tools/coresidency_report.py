#!/usr/bin/env python3
"""Summarises a rocprofv3 kernel trace of tools/coresidency_probe: for every concurrent repetition
(marked by the probe's k_delay kernel on the transfer stream), when the RCCL kernel started relative
to the gate and to the tree launches it had to share the GPU with.

    python tools/coresidency_report.py <run_kernel_trace.csv> [label]

Per repetition: `wait_us` = RCCL kernel start - k_delay end (the time the submitted transfer kernel
waited for CU resources; ~0 means it was admitted at once), `into_launch` = which tree launch was
running when it started and how far into it (a start near the end of a launch means it was admitted
only when that launch drained), `rccl_us` = its duration, `tree_span_us` = first tree start to last
tree end.  One JSON line per repetition plus a summary line.
"""
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else path
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"] = int(r["Start_Timestamp"]) / 1000.0
        r["e"] = int(r["End_Timestamp"]) / 1000.0
    rows.sort(key=lambda r: r["s"])
    delays = [r for r in rows if "k_delay" in r["Kernel_Name"]]
    out = []
    for d in delays:
        rccl = next((r for r in rows if r["s"] >= d["e"] - 1 and ("Generic" in r["Kernel_Name"]
                                                                   or "k_mimic" in r["Kernel_Name"])), None)
        trees = [r for r in rows if "k_reduce_tree" in r["Kernel_Name"] and d["s"] - 5 <= r["s"] <= d["s"] + 2000]
        if not rccl or not trees:
            continue
        # the tree launches of this repetition: consecutive ones from the gate on
        group = [trees[0]]
        for t in trees[1:]:
            if t["s"] - group[-1]["e"] > 20:
                break
            group.append(t)
        into = None
        for i, t in enumerate(group):
            if t["s"] <= rccl["s"] <= t["e"]:
                into = {"launch": i, "us_into": round(rccl["s"] - t["s"], 2), "launch_us": round(t["e"] - t["s"], 2)}
        rec = {
            "label": label,
            "wait_us": round(rccl["s"] - d["e"], 2),
            "gate_to_rccl_start_us": round(rccl["s"] - group[0]["s"], 2),
            "into_launch": into,
            "rccl_us": round(rccl["e"] - rccl["s"], 2),
            "rccl_grid": rccl.get("Grid_Size_X"), "rccl_wg": rccl.get("Workgroup_Size_X"),
            "rccl_lds": rccl.get("LDS_Block_Size"), "rccl_kernel": rccl["Kernel_Name"][:48],
            "tree_launches": len(group),
            "tree_span_us": round(group[-1]["e"] - group[0]["s"], 2),
            "tree_launch_us": [round(t["e"] - t["s"], 2) for t in group],
            "rccl_done_inside_tree_span": rccl["e"] <= group[-1]["e"],
        }
        out.append(rec)
        print(json.dumps(rec))
    if out:
        print(json.dumps({"label": label, "summary": True, "reps": len(out),
                          "median_wait_us": statistics.median(r["wait_us"] for r in out),
                          "median_rccl_us": statistics.median(r["rccl_us"] for r in out),
                          "median_tree_span_us": statistics.median(r["tree_span_us"] for r in out)}))


if __name__ == "__main__":
    main()
