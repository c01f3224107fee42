#!/usr/bin/env python3
"""Where the time of a multi-rank MPI test goes on the one-GPU box: runs one of the -m gpu suite's mpiexec command
lines (the reference's self-test mains or harnesses on the shim, every rank its own NCCL_HOSTID: RCCL's socket
transport) with RCCL's INIT / NET log on, and prints every output line with the seconds since launch, so that a slow
start (MPI, HIP, RCCL bootstrap, connection set-up) shows where it sits.  Measurement tooling only.

    python tools/mpi_timing.py selftest intra_scatter_radix_batch 8 2 4 3
    python tools/mpi_timing.py bin chiara_reduce_scatter 8 2 --overwrite b=4 base=1000 mem=device dtype=f32 reps=3
"""
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"


def main():
    kind, name, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    args = sys.argv[4:]
    exe = (os.path.join(REPO, "oracle", "_ref", f"selftest_{name}") if kind == "selftest" else
           os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd", "bin", name))
    debug = os.environ.get("NCCL_DEBUG", "INFO")
    cmd = [MPIEXEC]
    for r in range(n):
        if r:
            cmd.append(":")
        cmd += ["-n", "1", "-env", "NCCL_HOSTID", f"chiara-timing-{r}", "-env", "NCCL_SOCKET_IFNAME", "lo",
                "-env", "NCCL_IB_DISABLE", "1", "-env", "NCCL_DEBUG", debug, "-env", "NCCL_DEBUG_SUBSYS", "INIT,NET",
                exe] + args
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        p = subprocess.Popen(cmd, cwd=tmp, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        for line in p.stdout:
            print(f"{time.perf_counter() - t0:8.3f} {line.rstrip()[:200]}", flush=True)
        rc = p.wait()
    print(f"{time.perf_counter() - t0:8.3f} exit {rc}", flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
