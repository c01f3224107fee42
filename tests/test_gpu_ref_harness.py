"""Drop-in demonstration: the reference's OWN harnesses (Fugaku_experiments/Allreduce/main.cpp
and Reduce-scatter/main.cpp, compiled unchanged in the container into oracle/_ref/) linked
against libchiara through the reference-signature shim (csrc/shim/chiara_mpi_shim.cpp).
Their built-in is_correct (equality with MPI_Allreduce / MPI_Reduce_scatter_block on int32)
must be 1 on every row.  Likewise testing/main.cpp, the sweep of the six MPICH baselines
(check_correctness vs MPI_Allreduce on doubles, eps 1e-6).  4-5 MPI ranks share the test box's one GPU: each gets its own
NCCL_HOSTID so RCCL treats them as separate hosts."""
import csv
import os
import shutil
import subprocess

import pytest
from plot_pipeline import COLUMNS, per_algo_medians, plotter_frame

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
USEROP_SO = os.path.join(REPO, "tests", "userop", "libhalfadd_op.so")  # the user-op tests' device launchers
MPIEXEC = "/opt/conda/bin/mpiexec"


def _run(binary, args, n, tmp_path, where=("oracle", "_ref"), prefix="results", env=()):
    exe = os.path.join(REPO, *where, binary)
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("reference harness binary or MPICH not present")
    cmd = [MPIEXEC]
    for r in range(n):
        if r:
            cmd.append(":")
        cmd += ["-n", "1", "-env", "NCCL_HOSTID", f"chiara-ref-harness-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                "-env", "NCCL_IB_DISABLE", "1"]
        for kv in env:
            cmd += ["-env", *kv]
        cmd += [exe] + args
    out = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    files = [f for f in os.listdir(tmp_path) if f.startswith(prefix) and f.endswith(".csv")]
    assert len(files) == 1, files
    with open(os.path.join(tmp_path, files[0])) as f:
        return list(csv.DictReader(f))


def _plots(tmp_path, collective):
    """the CSV goes through the reference plotters' data stage unchanged."""
    path = [os.path.join(tmp_path, f) for f in os.listdir(tmp_path) if f.endswith(".csv")][0]
    with open(path) as f:
        assert f.readline().strip().split(",") == COLUMNS
    for agg in ("median", "min", "mean"):  # median_best / minimum_best / avg_best plotters
        wide, best, speedup = plotter_frame(path, collective, agg)
        assert best.notna().all().all() and (speedup > 0).all().all()


def test_reference_allreduce_harness_on_mi355x(tmp_path):
    rows = _run("ref_harness_allreduce", ["3", "--overwrite", "b=4", "base=64"], 4, tmp_path)
    ours = [r for r in rows if r["algorithm_name"] == "all_reduce_radix_batch"]
    assert len(ours) == 3 * 2 * 50  # n_iter x k in {2,3} x 50 reps
    assert {r["k"] for r in ours} == {"2", "3"}
    assert all(r["is_correct"] == "1" for r in rows)
    _plots(tmp_path, "allreduce")


def test_reference_harnesses_with_host_windows(tmp_path):
    """The shim turns pipelined host staging on: with 1 MiB windows (CHR_HOST_WINDOW_MIB) a 4 Mi-int
    call per rank runs as 4 window collectives, H2D / collective / D2H overlapped, the D2H from a
    second host thread.  The reference's own is_correct must still be 1 on every row."""
    (tmp_path / "ar").mkdir()
    rows = _run("ref_harness_allreduce", ["1", "--overwrite", "b=4", "base=1048576"], 4, tmp_path / "ar",
                env=[("CHR_HOST_WINDOW_MIB", "1")])
    assert {r["k"] for r in rows if r["algorithm_name"] == "all_reduce_radix_batch"} == {"2", "3"}
    assert all(r["is_correct"] == "1" for r in rows)
    (tmp_path / "rs").mkdir()
    rows = _run("ref_harness_reduce_scatter", ["1", "--overwrite", "b=4", "base=1048576"], 4, tmp_path / "rs",
                env=[("CHR_HOST_WINDOW_MIB", "1")])
    assert any(r["algorithm_name"] == "reduce_scatter_radix_batch" for r in rows)
    assert all(r["is_correct"] == "1" for r in rows)


def test_reference_reduce_scatter_harness_on_mi355x(tmp_path):
    rows = _run("ref_harness_reduce_scatter", ["2", "--overwrite", "b=4", "base=1000"], 4, tmp_path)
    ours = [r for r in rows if r["algorithm_name"] == "reduce_scatter_radix_batch"]
    assert len(ours) == 2 * 2 * 20
    assert all(r["is_correct"] == "1" for r in rows)
    _plots(tmp_path, "reduce_scatter")


def test_reference_mpich_baseline_harness_on_mi355x(tmp_path):
    """testing/main.cpp unchanged: every baseline, k = 2..nprocs-1, 50 reps per size."""
    rows = _run("ref_harness_testing", ["3", "--overwrite"], 5, tmp_path)
    names = {r["algorithm_name"] for r in rows}
    assert names == {"reduce_scatter_allgather_k", "recursive_exchange", "recursive_multiplying",
                     "reduce_scatter_allgather", "ring", "recursive_doubling"}
    assert len(rows) == 3 * (3 * 3 + 3) * 50  # sizes x (k in 2..4 x 3 + 3 without k) x reps
    assert {r["send_count"] for r in rows} == {"8", "16", "32"}
    assert all(r["is_correct"] == "1" for r in rows)


def test_reference_mpich_reduce_scatter_harness_on_mi355x(tmp_path):
    """testing/mpich_implementations/reduce_scatter/main.cpp unchanged: MPICH_reduce_scatter_radix at
    k = 2, 4, .., 30 (clamped to the 4 ranks), recursive halving, recursive doubling, pairwise and
    MPI_Reduce_scatter_block, 50 reps per size, check_correctness on doubles (eps 1e-9)."""
    rows = _run("ref_harness_rs_testing", ["2", "--overwrite"], 4, tmp_path, prefix="reduce_scatter_results")
    names = {r["algorithm_name"] for r in rows}
    assert names == {"MPICH_reduce_scatter_radix", "MPICH_reduce_scatter_rec_halving",
                     "MPICH_reduce_scatter_rec_doubling", "MPICH_reduce_scatter_pairwise", "MPI_Reduce_scatter_block"}
    assert len(rows) == 2 * (15 + 4) * 50  # sizes x (k = 2..30 step 2, four without k) x reps
    assert all(r["is_correct"] == "1" for r in rows)
    # the reference's per-algorithm plotter (make_median_algo_plot.py) accepts the CSV unchanged
    csvs = [f for f in os.listdir(tmp_path) if f.startswith("reduce_scatter_results")]
    med = per_algo_medians(os.path.join(tmp_path, csvs[0]))
    assert med["algorithm"].nunique() == 4 + 15 and (med["median_time"] > 0).all()


def test_reference_allgather_harness_on_mi355x(tmp_path):
    """Fugaku_experiments/Allgather/main.cpp unchanged: k = 2..b-1, check_correctness vs MPI_Allgather."""
    rows = _run("ref_harness_allgather", ["1", "--overwrite", "b=4", "base=16"], 8, tmp_path)
    ours = [r for r in rows if r["algorithm_name"] == "allgather_radix_batch"]
    assert ours and {r["k"] for r in ours} == {"2", "3"}
    assert all(r["is_correct"] == "1" for r in rows)
    _plots(tmp_path, "allgather")


@pytest.mark.parametrize("harness,algo", [("all_reduce", "all_reduce_radix_batch"),
                                          ("reduce_scatter", "reduce_scatter_radix_batch"),
                                          ("all_gather", "allgather_radix_batch")])
def test_reference_work_dir_harnesses_on_mi355x(tmp_path, harness, algo):
    """The development copies of the harnesses (testing/custom_implementations/work_dir/{all_reduce,
    reduce_scatter,all_gather}/main.cpp, 50 repetitions per size, their own CSV names), unchanged on the
    shim: every row is_correct, 4 ranks."""
    rows = _run(f"ref_harness_wd_{harness}", ["1", "--overwrite", "b=4", "base=64"], 4, tmp_path)
    assert any(r["algorithm_name"] == algo for r in rows)
    assert all(r["is_correct"] == "1" for r in rows)


BIN = ("configurable-hierarchical-allreduce-algorithms_amd", "bin")


# The reference's own harnesses above already cover the host-memory int32 path at 4 ranks with
# is_correct; these keep what only our harnesses add -- device-resident buffers (mem=device), f32 /
# bf16, 8 ranks -- at one case each (the plain-pattern f32 duplicates went).
# pattern=cancel: the reduced value is tiny next to sum|x_i|, so the association difference from MPI's
# own collective exceeds ulp(|result|); is_correct holds because the tolerance is (n-1)*ulp*sum|x_i|
# (harness_common.hpp check_correctness).  The device-resident allreduce and reduce-scatter run at 8 ranks
# (b = 4: two nodes of four, the C4 / C5 grouping), allgather and the host bf16 case at 4.
@pytest.mark.parametrize("binary,args,n,name,coll", [
    ("chiara_allreduce", ["2", "--overwrite", "b=4", "base=4096", "mem=device", "dtype=f32", "reps=3",
                          "pattern=cancel"], 8, "all_reduce_radix_batch", "allreduce"),
    ("chiara_reduce_scatter", ["2", "--overwrite", "b=4", "base=1000", "mem=device", "dtype=f32", "reps=3",
                               "pattern=cancel"], 8, "reduce_scatter_radix_batch", "reduce_scatter"),
    ("chiara_allgather", ["2", "--overwrite", "b=4", "base=100", "mem=device", "dtype=bf16", "reps=3"], 4,
     "allgather_radix_batch", "allgather"),
    ("chiara_allreduce", ["2", "--overwrite", "b=4", "base=1000", "mem=host", "dtype=bf16", "reps=3",
                          "pattern=cancel"], 4, "all_reduce_radix_batch", "allreduce"),
])
def test_own_harnesses_device_resident(tmp_path, binary, args, n, name, coll):
    """csrc/harness: the reference CLI/CSV with the HBM-resident extension (mem=device)."""
    rows = _run(binary, args, n, tmp_path, where=BIN)
    ours = [r for r in rows if r["algorithm_name"] == name]
    bad = [r for r in rows if r["is_correct"] != "1"]
    assert ours and not bad, bad[:5]
    if "dtype=bf16" not in args or coll == "allgather":  # MPI has no bf16: no baseline rows to plot against
        _plots(tmp_path, coll)


def test_shim_over_mpi_datatype_op_table(tmp_path):
    """The reference-signature binding (csrc/shim) on every MPI predefined datatype x op, the MAXLOC /
    MINLOC pair types and the C complex types included: pairs MPICH's MPI_Reduce_local accepts give
    MPI_Allreduce's / MPI_Reduce_scatter_block's result through all_reduce_radix_batch,
    reduce_scatter_radix_batch and MPICH_Allreduce_ring (complex by value: a zero part's sign follows
    the association); pairs it rejects, user ops, the long-double types and non-contiguous allgather
    types come back as MPI error classes (shim_types_main.cpp).  User ops bound to device launchers
    (chiara_shim_op_bind, tests/userop/libhalfadd_op.so): a commutative one equals MPI's own collectives, a
    non-commutative one is refused by k-reduce-scatter-allgather with MPI_ERR_OP, as the reference refuses it."""
    import json

    exe = os.path.join(REPO, *BIN, "chiara_shim_types")
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("shim types binary or MPICH not present")
    cmd = [MPIEXEC]
    for r in range(4):
        if r:
            cmd.append(":")
        cmd += ["-n", "1", "-env", "NCCL_HOSTID", f"chiara-shim-types-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                "-env", "NCCL_IB_DISABLE", "1", "-env", "CHR_SHIM_USEROP_SO", USEROP_SO, exe]
    out = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=400)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(line[-1])
    assert out.returncode == 0 and res["failures"] == 0, res
    # 31 types x 12 ops; MPICH accepts 226 of the pairs (the MAXLOC / MINLOC pair types and the C
    # complex types included)
    assert res["pairs"] == 372 and res["supported_by_mpich"] >= 226, res
    # user ops bound to their device launchers through the shim (chiara_shim_op_bind): checked
    assert res["userop"] == 1, res


# One geometry per self-test main (each run starts n MPI processes, each with HIP and an RCCL
# communicator): intra_reduce_scatter with step-1 folds (b = 3, k = 2), inter_linear_reduce with a leftover
# iteration (nnodes = 3, b = 2), intra_scatter with a two-level k-nomial tree (k = 2, b = 4), and the DEBUG
# mains of all_reduce_radix_batch.cpp and of the MPICH baselines at 6 ranks (non-power-of-two folds).
# tests/golden/selftest_outputs.json holds more phase geometries, checked against the oracle on CPU.
SELFTEST_RUNS = ("intra_reduce_scatter_radix_n9_2_2_3", "inter_linear_reduce_n6_2_3", "intra_scatter_radix_batch_n8_2_4_3",
                 "all_reduce_radix_batch_n6_3_b2", "reduce_scatter_radix_n6_3", "reduce_scatter_recursive_halving_n6_2_2",
                 "reduce_scatter_pairwise_n6_", "allreduce_ring_n6_", "allreduce_recursive_doubling_n6_",
                 "allreduce_reduce_scatter_allgather_n6_", "allreduce_recexch_n6_", "allreduce_k_reduce_scatter_allgather_n6_",
                 "allreduce_recursive_multiplying_n6_")


def _selftest_cases():
    import json

    with open(os.path.join(REPO, "tests", "golden", "selftest_outputs.json")) as f:
        runs = json.load(f)["runs"]
    return [(k, runs[k]) for k in SELFTEST_RUNS]


@pytest.mark.parametrize("name,run", _selftest_cases(), ids=list(SELFTEST_RUNS))
def test_reference_selftests_on_mi355x(tmp_path, name, run):
    """The reference's DEBUG_MODE self-test mains, each compiled unchanged with -DDEBUG_MODE
    (oracle/selftests.sh) with its algorithm function replaced through the shim by libchiara's: CHiArA's
    stand-alone phases, all_reduce_radix_batch.cpp and the MPICH baselines.  Every rank prints exactly the
    lines the reference's own build printed here, and writes the same files (tests/golden/selftest_outputs.json,
    normalised by tests/selftest_util.py: wall-clock times masked) -- every PASS line, is_correct column and
    printed buffer included."""
    import selftest_util

    exe = os.path.join(REPO, "oracle", "_ref", f"selftest_{run['binary']}")
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("self-test binary or MPICH not present")
    n = run["nranks"]
    fn = selftest_util.shim_functions()[run["binary"]]
    cmd = [MPIEXEC, "-outfile-pattern", "out.%r", "-errfile-pattern", "err.%r"]
    for r in range(n):
        if r:
            cmd.append(":")
        cmd += ["-n", "1", "-env", "NCCL_HOSTID", f"chiara-selftest-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                "-env", "NCCL_IB_DISABLE", "1", "-env", "CHR_SHIM_TRACE", "1", exe] + run["args"]
    out = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    errs = {r: (tmp_path / f"err.{r}").read_text(encoding="utf-8") if (tmp_path / f"err.{r}").exists() else ""
            for r in range(n)}
    assert out.returncode == 0, out.stderr[-3000:] + "".join(errs.values())[-3000:]
    for r in range(n):
        # the positive marker: this rank's calls went through the shim's definition of the function
        # (CHR_SHIM_TRACE), not through the reference file's own, which the build only weakened
        calls = selftest_util.shim_calls(errs[r])
        assert calls is not None and calls[0] == r and calls[1].get(fn, 0) >= 1, (r, fn, errs[r][-2000:])
        raw = (tmp_path / f"out.{r}").read_text(encoding="utf-8") if (tmp_path / f"out.{r}").exists() else ""
        # the reference function's own DEBUG_MODE phase timers must be absent (they would mean its body ran)
        assert not selftest_util.reference_phase_lines(raw), (r, selftest_util.reference_phase_lines(raw)[:3])
        got = selftest_util.normalize(raw)
        assert got == run["lines"][str(r)], (r, got, run["lines"][str(r)])
    for fname, want in run.get("files", {}).items():
        text = (tmp_path / fname).read_text(encoding="utf-8")
        got = selftest_util.normalize_csv(text) if fname.endswith(".csv") else text.splitlines()
        assert got == want, (fname, got[:10], want[:10])
