#!/usr/bin/env python3
"""Holds HIP hardware queues the way the -m gpu suite's pytest process does after its in-process tests (torch's
streams, a local group's streams, one RCCL communicator), then sleeps: the background process of an A/B on whether
a GPU-holding parent slows the multi-rank MPI / RCCL children the suite starts.  Measurement
tooling only.

    python3 tools/hold_queues.py SECONDS"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402

import chiara_amd as ca  # noqa: E402


def main():
    secs = float(sys.argv[1])
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    x = torch.ones(1 << 20, device=dev)
    for s in streams:
        with torch.cuda.stream(s):
            x.add_(1.0)
    g = ca.LocalGroup(8, 0)
    sends = [torch.ones(8 * 4096, device=dev) for _ in range(8)]
    recvs = [torch.empty_like(t) for t in sends]
    ca.check(g.all_reduce_radix_batch(sends, recvs, 8 * 4096, ca.FLOAT32, ca.SUM, 4, 4))
    comm = ca.Comm(1, ca.get_unique_id(), 0, 0)
    ca.check(ca.all_reduce_radix_batch(sends[0], recvs[0], 8 * 4096, ca.FLOAT32, ca.SUM, comm, 2, 1))
    torch.cuda.synchronize()
    print("holding", flush=True)
    time.sleep(secs)
    comm.destroy()
    g.destroy()
    print("released", flush=True)


if __name__ == "__main__":
    main()
