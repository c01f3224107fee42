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
