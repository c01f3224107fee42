import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")
for p in (REPO, PKG_DIR, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


_DURATIONS = []
# The driver's -m gpu step is killed at 900 s, and a timed-out suite would leave every parity row untested: the calls
# of the whole GPU suite must sum to at most this.  Over it, the summary warns; with
# CHR_GPU_SUITE_BUDGET_STRICT=1 (tools/gpu.sh suite sets it) the run fails, so a builder run that grows the suite
# past the budget is caught before the driver's is.
GPU_SUITE_BUDGET_S = 420


def pytest_runtest_logreport(report):
    if report.when == "call" or (report.when == "setup" and report.failed):
        _DURATIONS.append((report.duration, report.nodeid))


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Per-test durations in the run's log, the slowest first, and the total against the GPU suite's
    time budget."""
    if not _DURATIONS:
        return
    total = sum(d for d, _ in _DURATIONS)
    tr = terminalreporter
    tr.write_sep("-", f"chiara test durations: {len(_DURATIONS)} tests, {total:.1f} s in calls")
    for d, nodeid in sorted(_DURATIONS, reverse=True)[:15]:
        tr.write_line(f"{d:8.2f}s  {nodeid}")
    if over_budget(config):
        tr.write_line(f"WARNING: the GPU suite took {total:.0f} s, over its {GPU_SUITE_BUDGET_S} s budget")


def over_budget(config):
    return getattr(config.option, "markexpr", "") == "gpu" and sum(d for d, _ in _DURATIONS) > GPU_SUITE_BUDGET_S


def pytest_sessionfinish(session, exitstatus):
    if os.environ.get("CHR_GPU_SUITE_BUDGET_STRICT") == "1" and over_budget(session.config) and exitstatus == 0:
        session.exitstatus = 1


# GPU tests whose GPU work runs only in child processes (mpiexec ranks, spawned RCCL ranks, per-configuration kernel
# children, the two-process IPC probe) run first, before this process's own tests touch the GPU: with a process that
# holds HIP streams, a local group and an RCCL communicator alive beside them, an 8-rank self-test main took 34-38 s
# and an 8-rank harness 21-23 s, against 4-9 s and 5 s without (tools/hold_queues.py, profiles/r06/mpi_timing/) --
# which is where the suite's 8-rank cases lost their time.
CHILD_ONLY_GPU_TESTS = ("tests/test_gpu_ref_harness.py::", "tests/test_gpu_rccl_multirank.py::",
                        "tests/test_gpu_xcd_map.py::", "tests/test_gpu_ipc.py::test_hip_ipc_handle_between_two_processes")


def pytest_collection_modifyitems(session, config, items):
    first = [it for it in items if it.nodeid.startswith(CHILD_ONLY_GPU_TESTS)]
    ids = {id(it) for it in first}
    items[:] = first + [it for it in items if id(it) not in ids]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_mpich():
    """Golden vectors of the MPICH baselines testing/main.cpp drives (gen_golden.py mpich)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "mpich_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "mpich_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_types():
    """Golden vectors of the integer types beyond int32 and the logical/bitwise ops, from the
    reference compiled here against MPICH (gen_golden.py types)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "types_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "types_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_pairtypes():
    """Golden vectors of MPI's pair types (MAXLOC / MINLOC) and the C complex types (SUM / PROD) from
    the reference compiled here, or MPI's own collective where the reference cannot address the
    type (gen_golden.py pairs; modes ar_lib / rs_lib).  Outputs are stored as raw bytes."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "pairtypes_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "pairtypes_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_rsmpich():
    """Golden vectors of the MPICH baseline reduce-scatters that
    testing/mpich_implementations/reduce_scatter/main.cpp drives (gen_golden.py rsmpich)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "rsmpich_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "rsmpich_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_phases():
    """Golden vectors of CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/
    reduce_scatter/{intra_reduce_scatter_radix, inter_linear_reduce, intra_scatter_radix_batch}.cpp, compiled
    unchanged against MPICH; gen_golden.py phases)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "phases_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "phases_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays
