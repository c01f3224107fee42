"""SURVEY §8(f) row 4, CSV / plot parity, CPU side: the restated data stage of the reference's
plotters (tests/plot_pipeline.py) is pinned on samples of the reference's own result CSVs
(tests/golden/plot_samples/, cut by gen_samples.py), and refuses what the plotters refuse.  The
GPU side (tests/test_gpu_ref_harness.py) puts the CSVs the harnesses write on MI355X through it."""
import os

import pandas as pd
import pytest

from plot_pipeline import BASELINES, COLUMNS, per_algo_medians, plotter_frame

SAMPLES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "plot_samples")


@pytest.mark.parametrize("collective", sorted(BASELINES))
@pytest.mark.parametrize("agg", ["median", "min", "mean"])
def test_reference_csv_samples(collective, agg):
    path = os.path.join(SAMPLES, f"{collective}.csv")
    with open(path) as f:
        assert f.readline().strip().split(",") == COLUMNS
    wide, best, speedup = plotter_frame(path, collective, agg)
    assert BASELINES[collective] in wide.columns
    assert len(wide.columns) >= 2 and best.notna().all().all()
    assert (speedup > 0).all().all()


def _write(tmp_path, rows):
    p = os.path.join(tmp_path, "results.csv")
    pd.DataFrame(rows, columns=COLUMNS).to_csv(p, index=False)
    return p


def test_refuses_incorrect_rows(tmp_path):
    p = _write(tmp_path, [["MPICH_allreduce", 0, 0, 8, 128, 1e-4, 1],
                          ["all_reduce_radix_batch", 2, 4, 8, 128, 5e-5, 0]])
    with pytest.raises(RuntimeError, match="incorrect"):
        plotter_frame(p, "allreduce")


def test_requires_baseline(tmp_path):
    p = _write(tmp_path, [["all_reduce_radix_batch", 2, 4, 8, 128, 5e-5, 1]])
    with pytest.raises(RuntimeError, match="Baseline"):
        plotter_frame(p, "allreduce")


def test_k_labels_and_speedup(tmp_path):
    """k > 0 rows are labelled per k; the speedup is baseline / best of the others (:49-56)."""
    p = _write(tmp_path, [["MPICH_allreduce", 0, 0, 8, 128, 4e-4, 1],
                          ["all_reduce_radix_batch", 2, 4, 8, 128, 2e-4, 1],
                          ["all_reduce_radix_batch", 4, 4, 8, 128, 1e-4, 1],
                          ["all_reduce_radix_batch", 4, 4, 8, 128, 3.5e-4, 1]])
    wide, best, speedup = plotter_frame(p, "allreduce")
    assert set(wide.columns) == {"MPICH_allreduce", "all_reduce_radix_batch (k=2)", "all_reduce_radix_batch (k=4)"}
    assert best.loc[8, 128] == "all_reduce_radix_batch (k=2)"  # k=4: median 2.25e-4
    assert speedup.loc[8, 128] == pytest.approx(2.0)


def test_reference_mpich_reduce_scatter_sample_per_algo_medians():
    """make_median_algo_plot.py on the reference's own MPICH reduce-scatter baseline results: every
    radix k is its own line, the k-less baselines keep their names."""
    med = per_algo_medians(os.path.join(SAMPLES, "reduce_scatter_mpich.csv"))
    algos = set(med["algorithm"])
    assert {"MPICH_reduce_scatter_pairwise", "MPICH_reduce_scatter_rec_doubling", "MPICH_reduce_scatter_rec_halving",
            "MPI_Reduce_scatter_block"} <= algos
    assert {f"MPICH_reduce_scatter_radix (k={k})" for k in range(2, 32, 2)} <= algos
    assert (med["median_time"] > 0).all() and med["send_count_norm"].nunique() == 2


def test_per_algo_medians_refuses_incorrect_rows(tmp_path):
    p = _write(tmp_path, [["MPICH_reduce_scatter_pairwise", 0, 0, 4, 32, 1e-4, 0]])
    with pytest.raises(RuntimeError, match="incorrect"):
        per_algo_medians(p)
