#!/usr/bin/env python3
"""Message traces of the REAL reference collectives (container-only).

Builds oracle/_ref/ref_trace (the reference's allreduce / reduce-scatter files compiled
unchanged against the container's MPICH 3.3.2, point-to-point calls intercepted through
PMPI) and records, for every rank of every geometry, the ordered list of
(direction, peer, bytes) it posts.  Writes tests/golden/msg_trace.json, which pins the
communication pattern of libchiara's `exact` schedule (tests/test_exact_schedule.py).
Rerun: python tests/golden/gen_trace.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle")
MPIEXEC = "/opt/conda/bin/mpiexec"
RC = 3  # recvcount (elements per rank block); fp32


def divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def geometries():
    for n in (2, 3, 4, 5, 6, 8, 9, 12, 16):
        for b in divisors(n):
            for k in (2, 3, 4, 5, 8):
                if k > max(b, 2) + 1 and k != 2:
                    continue  # k clamps to b (all_reduce_radix_batch.cpp:19-21); one clamp probe kept
                yield n, k, b


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "ref_trace"])
    exe = os.path.join(ORACLE, "_ref", "ref_trace")
    cases = []
    for n, k, b in geometries():
        for mode in ("ar", "rs"):
            count = RC * n if mode == "ar" else RC
            cmd = [MPIEXEC, "-n", str(n)]
            if n <= os.cpu_count():
                cmd[1:1] = ["-bind-to", "core"]
            out = subprocess.run(cmd + [exe, mode, str(k), str(b), str(count)], capture_output=True, text=True,
                                 timeout=120, check=True).stdout
            ranks = [None] * n
            for line in out.strip().splitlines():
                r = json.loads(line)
                ranks[r["rank"]] = r["msgs"]
            cases.append({"mode": mode, "n": n, "k": k, "b": b, "count": count, "elem_bytes": 4, "ranks": ranks})
    with open(os.path.join(HERE, "msg_trace.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_trace.py (oracle/ref_trace.cpp, MPICH 3.3.2 PMPI)",
                   "format": "ranks[r] = ordered [dir (0 send, 1 recv), peer, bytes] posted by rank r",
                   "cases": cases}, f, separators=(",", ":"))
    print(f"{len(cases)} traces")


if __name__ == "__main__":
    main()
