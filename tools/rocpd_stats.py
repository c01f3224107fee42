#!/usr/bin/env python3
"""Summarise a rocprofv3 database (rocpd .db, the ROCm 7.2 default output) as the `--stats` kernel
CSV: per kernel name the calls, total / average / min / max duration in microseconds, plus the
average over the LAST k dispatches of each kernel (the timed region of bench.py, after warmup).
Usage: rocpd_stats.py <results.db> [--last K] [--csv out.csv]"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels order by start"):
        rows.setdefault(name, []).append(dur / 1e3)  # ns -> us
    out = []
    for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        rec = {"name": name, "calls": len(d), "total_us": round(sum(d), 3), "avg_us": round(sum(d) / len(d), 4),
               "min_us": round(min(d), 4), "max_us": round(max(d), 4)}
        if a.last:
            tail = d[-a.last:]
            rec[f"avg_last{a.last}_us"] = round(sum(tail) / len(tail), 4)
        out.append(rec)
    w = csv.DictWriter(open(a.csv, "w", newline="") if a.csv else sys.stdout, fieldnames=list(out[0].keys()))
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()
