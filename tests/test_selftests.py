"""The reference's DEBUG_MODE self-test mains as built against the reference itself
(tests/golden/selftest_outputs.json, oracle/selftests.sh): their own verdicts are all passes, so the GPU test
that runs the same mains on libchiara (tests/test_gpu_ref_harness.py::test_reference_selftests_on_mi355x) and
requires identical output requires passes too.  Also the normaliser masks only wall-clock times."""
import json
import os

import selftest_util

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _runs():
    with open(os.path.join(HERE, "selftest_outputs.json")) as f:
        return json.load(f)["runs"]


def test_reference_selftests_report_passes():
    runs = _runs()
    mains = {r["binary"] for r in runs.values()}
    assert len(mains) == 13, sorted(mains)
    for key, run in runs.items():
        text = "\n".join(ln for lines in run["lines"].values() for ln in lines)
        assert "FAIL" not in text and "mismatch" not in text.lower() and "❌" not in text, key
        if run["binary"] in ("reduce_scatter_radix", "reduce_scatter_pairwise"):
            assert "✅ All tests passed" in text, key
        if run["binary"].startswith("allreduce_"):
            assert "PASSED" in text, key
        if run["binary"] == "all_reduce_radix_batch":
            rows = run["files"]["results0.csv"][1:]
            assert len(rows) == 2 * 3 and all(r.endswith(",1") for r in rows), rows  # 2 reps x 3 sizes, is_correct
        if run["binary"] == "reduce_scatter_recursive_halving":
            assert any(ln.startswith("SendRank") for ln in run["files"]["all_buffers.txt"]), key


def test_normalize_masks_times_only():
    text = ("RCCL version : 2.27.7\nRing implementation: PASSED, Time: 0.000049114 seconds\n"
            "Red-Scatter Phase 1 time: 0.000012\nTest PASSED: All 10 values match\n"
            "Performance Summary:\nk=2: 0.1 seconds (fastest so far)\n")
    assert selftest_util.normalize(text) == ["Ring implementation: PASSED, Time: <t> seconds",
                                             "Test PASSED: All 10 values match"]
    assert selftest_util.normalize_csv("algorithm_name,time,is_correct\nx,0.5,1\n") == [
        "algorithm_name,time,is_correct", "x,<t>,1"]


def test_build_recipe_and_gpu_runs_match_the_goldens():
    """oracle/selftests.sh builds every main the goldens hold, and every run the GPU test starts has a golden."""
    import re
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(os.path.dirname(here), "oracle", "selftests.sh")) as f:
        specs = re.search(r"<<'SPECS'\n(.*?)\nSPECS", f.read(), re.S).group(1).split("\n")
    built = {ln.split()[0] for ln in specs if ln.strip()}
    runs = _runs()
    assert {r["binary"] for r in runs.values()} == built
    sys.path.insert(0, here)
    src = open(os.path.join(here, "test_gpu_ref_harness.py")).read()
    gpu_runs = re.search(r"SELFTEST_RUNS = \((.*?)\)\n", src, re.S).group(1)
    keys = re.findall(r'"([^"]+)"', gpu_runs)
    assert keys and all(k in runs for k in keys)
    assert {runs[k]["binary"] for k in keys} == built  # one GPU run per main


# ---- the shim-linked self-test binaries really bind to the shim -------------------

import re  # noqa: E402
import shutil  # noqa: E402
import subprocess  # noqa: E402

import pytest  # noqa: E402

REF_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref")
_CALL = re.compile(r"\bcall\s+[0-9a-f]+\s+<([^>]+)>")


def _defined(exe, fn):
    """Defined text symbols of `exe` for the C++ function `fn` (mangled prefix _Z<len><fn>)."""
    out = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    pre = f"_Z{len(fn)}{fn}"
    return [f[2] for f in (ln.split() for ln in out.splitlines()) if len(f) == 3 and f[1] in "TtWw"
            and f[2].startswith(pre)]


def _calls(exe, sym):
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", f"--disassemble={sym}", exe], capture_output=True,
                         text=True, check=True).stdout
    return _CALL.findall(out)


def _reaches_libchiara(exe, sym, depth=2):
    """True when `sym`'s body -- or a function it calls directly inside the binary, to `depth` levels --
    calls one of libchiara's chr_* entry points through the PLT."""
    calls = _calls(exe, sym)
    if any(c.startswith("chr_") and c.endswith("@plt") for c in calls):
        return True
    return depth > 0 and any(_reaches_libchiara(exe, c, depth - 1) for c in calls
                             if "@plt" not in c and "+" not in c)


def _binding(exe, fn):
    syms = _defined(exe, fn)
    strong = [s for s in syms if s in _strong_text(exe)]
    return strong, bool(strong) and len(strong) == 1 and _reaches_libchiara(exe, strong[0])


def _strong_text(exe):
    out = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    return {f[2] for f in (ln.split() for ln in out.splitlines()) if len(f) == 3 and f[1] == "T"}


def _need_tools():
    if not (shutil.which("nm") and shutil.which("objdump")):
        pytest.skip("binutils absent")


@pytest.mark.parametrize("name", sorted(selftest_util.shim_functions()))
def test_selftest_binary_binds_function_to_shim(name):
    """Each oracle/_ref/selftest_<name> defines the replaced function exactly once, as a global text symbol,
    and that definition calls into libchiara (chr_*@plt) -- so its main, whose call is a relocation against
    the symbol (-fno-inline), runs the shim.  The reference-only build (selftest_<name>_mpi, the negative
    control) defines it too, and never reaches libchiara: the check can fail."""
    _need_tools()
    fn = selftest_util.shim_functions()[name]
    exe, ctl = os.path.join(REF_DIR, f"selftest_{name}"), os.path.join(REF_DIR, f"selftest_{name}_mpi")
    if not os.path.exists(exe) or not os.path.exists(ctl):
        pytest.skip("self-test binaries not built (oracle/selftests.sh, container-only)")
    strong, ok = _binding(exe, fn)
    assert ok, (name, fn, strong)
    strong_ctl, ok_ctl = _binding(ctl, fn)
    assert len(strong_ctl) == 1 and not ok_ctl, (name, strong_ctl)


def test_gpu_selftest_checks_reject_the_reference_only_build(tmp_path):
    """Negative control for test_gpu_ref_harness.py::test_reference_selftests_on_mi355x, on CPU: the
    reference-only build of all_reduce_radix_batch.cpp's DEBUG main (selftest_*_mpi: its own function, no
    shim), run exactly as the GPU test runs the shim build (CHR_SHIM_TRACE=1, one output file per rank),
    fails both of that test's binding checks -- no shim marker on stderr, and the function's own
    `Phase N time:` lines in the output -- while its normalised lines still equal the golden ones (which is
    why the normaliser alone could not tell the builds apart)."""
    mpiexec = "/opt/conda/bin/mpiexec"
    exe = os.path.join(REF_DIR, "selftest_all_reduce_radix_batch_mpi")
    if not (os.path.exists(exe) and os.path.exists(mpiexec)):
        pytest.skip("reference self-test build or MPICH absent (container-built)")
    run = _runs()["all_reduce_radix_batch_n6_3_b2"]
    n = run["nranks"]
    out = subprocess.run([mpiexec, "-outfile-pattern", "out.%r", "-errfile-pattern", "err.%r", "-n", str(n),
                          "-env", "CHR_SHIM_TRACE", "1", exe] + run["args"], cwd=tmp_path, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    phases = []
    for r in range(n):
        err = (tmp_path / f"err.{r}").read_text() if (tmp_path / f"err.{r}").exists() else ""
        raw = (tmp_path / f"out.{r}").read_text() if (tmp_path / f"out.{r}").exists() else ""
        assert selftest_util.shim_calls(err) is None
        assert selftest_util.normalize(raw) == run["lines"][str(r)]
        phases.append(bool(selftest_util.reference_phase_lines(raw)))
    assert phases[0], "rank 0 prints the reference function's phase timers"
