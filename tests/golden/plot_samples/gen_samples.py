"""Cut small samples of the reference's own benchmark CSVs (testing/plots/*, data files) into
tests/golden/plot_samples/ for tests/test_plot_pipeline.py.  Container-only: reads /root/reference."""
import os

import pandas as pd

SRC = "/root/reference/testing/plots"
HERE = os.path.dirname(os.path.abspath(__file__))
for name, rel in (("allreduce", "all_reduce/results_custom_polaris.csv"),
                  ("reduce_scatter", "reduce_scatter/results_polaris_final.csv"),
                  ("allgather", "all_gather/results_fugaku_48_final.csv")):
    df = pd.read_csv(os.path.join(SRC, rel)).dropna(subset=["algorithm_name"])
    df = df[df["nprocs"] == sorted(df["nprocs"].unique())[0]]
    sizes = sorted(df["send_count"].unique())[:3]
    df = df[df["send_count"].isin(sizes)]
    df.to_csv(os.path.join(HERE, f"{name}.csv"), index=False)
    print(name, len(df), "rows", sorted(df["algorithm_name"].unique()))

# the MPICH reduce-scatter baselines' own results (testing/mpich_implementations/reduce_scatter/,
# the CSV make_median_algo_plot.py reads): two sizes of the 8-rank file
df = pd.read_csv("/root/reference/testing/mpich_implementations/reduce_scatter/reduce_scatter_results8.csv")
sizes = sorted(df["send_count"].unique())[:2]
df = df[df["send_count"].isin(sizes)]
df.to_csv(os.path.join(HERE, "reduce_scatter_mpich.csv"), index=False)
print("reduce_scatter_mpich", len(df), "rows", sorted(df["algorithm_name"].unique()))
