"""The data stage of the reference's plotters, restated (test infrastructure).

testing/plots/all_reduce/median_best_plotter.py:12-56, reduce_scatter/median_best_plotter.py and
minimum_best_plotter.py, all_gather/median_best_plotter.py and avg_best_plotter.py all do the same
before drawing: read the CSV, refuse any row with is_correct != 1 (:15-20), label each algorithm
with its k when k > 0 (:23-26), aggregate time per (nprocs, send_count, algorithm) (:29-33),
pivot to one column per algorithm (:36), require the baseline column (:39-41: MPICH_allreduce,
reduce_scatter_standard, allgather_standard), pick the per-cell winner (:45) and the speedup of the
best non-baseline algorithm over the baseline (:49-56).  matplotlib is absent here, so only this
stage runs; it is what decides whether a CSV is consumable by the plotters unchanged.

testing/plots/reduce_scatter/make_median_algo_plot.py (the per-algorithm view used for the MPICH
reduce-scatter baselines' CSVs, testing/mpich_implementations/reduce_scatter/) has a data stage of
its own, restated in per_algo_medians.
"""
import pandas as pd

BASELINES = {"allreduce": "MPICH_allreduce", "reduce_scatter": "reduce_scatter_standard",
             "allgather": "allgather_standard"}
COLUMNS = ["algorithm_name", "k", "b", "nprocs", "send_count", "time", "is_correct"]


def plotter_frame(csv_path, collective, agg="median"):
    """Returns (wide, best_algo, speedup) exactly as the plotters compute them; raises
    RuntimeError where the plotters raise."""
    df = pd.read_csv(csv_path)
    if not df["is_correct"].eq(1).all():
        bad = df.loc[df["is_correct"] != 1, ["nprocs", "send_count", "algorithm_name", "k", "time"]]
        raise RuntimeError(f"Found {len(bad)} incorrect measurement(s)")
    df["algorithm"] = df.apply(
        lambda r: f"{r['algorithm_name']} (k={int(r['k'])})" if r["k"] > 0 else r["algorithm_name"], axis=1)
    g = df.groupby(["nprocs", "send_count", "algorithm"])["time"]
    med = getattr(g, agg)().reset_index()
    wide = med.pivot(index=["nprocs", "send_count"], columns="algorithm", values="time")
    base = BASELINES[collective]
    if base not in wide.columns:
        raise RuntimeError(f"Baseline '{base}' not found in data: {list(wide.columns)}")
    best_algo = wide.idxmin(axis=1).unstack(level=-1)
    mine = [c for c in wide.columns if c != base]
    if not mine:
        raise RuntimeError("No non-baseline algorithms found to compare against the baseline.")
    speedup = (wide[base] / wide[mine].min(axis=1)).unstack(level=-1)
    return wide, best_algo, speedup


def per_algo_medians(csv_path):
    """make_median_algo_plot.py's data stage: refuse incorrect rows (:25-32) and missing columns
    (:34-37), label variants by k when k is set and nonzero (:40-44), x = send_count / nprocs
    (:47), median time per (nprocs, x, algorithm) (:50-55).  Returns that frame."""
    df = pd.read_csv(csv_path)
    if "is_correct" in df.columns and not df["is_correct"].eq(1).all():
        raise RuntimeError("Found incorrect measurement(s)")
    need = {"nprocs", "send_count", "algorithm_name", "k", "time"}
    miss = need - set(df.columns)
    if miss:
        raise RuntimeError(f"Missing columns: {sorted(miss)}")
    df["algorithm"] = df.apply(
        lambda r: f"{r['algorithm_name']} (k={int(r['k'])})" if pd.notna(r["k"]) and int(r["k"]) != 0
        else str(r["algorithm_name"]), axis=1)
    df["send_count_norm"] = df["send_count"] / df["nprocs"]
    return (df.groupby(["nprocs", "send_count_norm", "algorithm"], as_index=False)["time"].median()
            .rename(columns={"time": "median_time"}))
