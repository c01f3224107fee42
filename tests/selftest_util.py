"""Normalisation of the reference's DEBUG_MODE self-test output (tests/golden/gen_selftests.py writes the
reference build's, tests/test_gpu_ref_harness.py compares the shim build's).  What is dropped or masked is
what differs between two runs of the SAME program, or what only the reference's function prints:
* RCCL's rank-0 banner ("RCCL version : ...", "Librccl path : ...") and NCCL/RCCL log lines;
* the phase timers the reference's all_reduce_radix_batch prints under DEBUG_MODE (its function is the one
  the shim replaces: all_reduce_radix_batch.cpp:256-349);
* wall-clock numbers on lines that report a time, and recursive multiplying's "Performance Summary"
  ranking of those times (allreduce_recursive_multiplying.cpp's main).
Every check line -- PASS / FAILED / mismatch / the printed buffers -- is kept verbatim.

The shim-linked runs are also checked positively: the shim's CHR_SHIM_TRACE line must
name the replaced function on every rank, and the reference function's phase timers must be absent from the
raw output -- a build whose call bound back to the reference's own function fails both checks."""
import os
import re

_SPECS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "selftests.sh")
_SHIM_LINE = re.compile(r"^\[chiara-shim\] rank (\d+) calls:(.*)$", re.M)
_PHASE = re.compile(r"Phase \d+ time:")


def shim_functions():
    """{self-test name: the reference function the shim replaces in it}, from oracle/selftests.sh's table."""
    text = open(_SPECS, encoding="utf-8").read()
    body = text.split("<<'SPECS'\n", 1)[1].split("\nSPECS", 1)[0]
    return {f[0]: f[2] for f in (ln.split() for ln in body.splitlines()) if len(f) == 3}


def shim_calls(stderr_text):
    """(rank, {function: calls}) from the shim's CHR_SHIM_TRACE exit line, or None if it is absent."""
    m = _SHIM_LINE.findall(stderr_text)
    if not m:
        return None
    rank, rest = m[-1]
    return int(rank), {k: int(v) for k, v in (t.split("=", 1) for t in rest.split())}


def reference_phase_lines(text):
    return [ln for ln in text.splitlines() if _PHASE.search(ln)]

_NUM = re.compile(r"\d+\.\d+(?:e[-+]?\d+)?")


def normalize(text):
    out = []
    for ln in text.splitlines():
        ln = ln.rstrip()
        if " : " in ln or "NCCL " in ln:
            continue
        if re.search(r"Phase \d+ time:", ln):
            continue
        if "Performance Summary" in ln:
            break
        if re.search(r"[Tt]ime|seconds", ln):
            ln = _NUM.sub("<t>", ln)
        out.append(ln)
    return out


def normalize_csv(text):
    """A results CSV (algorithm_name,k,b,nprocs,send_count,time,is_correct): the time column masked."""
    rows = [ln.split(",") for ln in text.splitlines() if ln.strip()]
    if not rows:
        return []
    t = rows[0].index("time") if "time" in rows[0] else None
    return [",".join("<t>" if (i == t and r is not rows[0]) else v for i, v in enumerate(r)) for r in rows]
