#!/usr/bin/env python3
"""Runs tools/coresidency_probe.cpp (built as tools/libcoresidency_probe.so) inside a Python process
after `import torch`, so its RCCL calls go to torch's bundled RCCL -- the library bench.py's N>1
line and every torch.distributed bootstrap use -- instead of ROCm 7.2's.  Arguments are the probe's.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]

import torch  # noqa: E402,F401  (loads torch's libamdhip64 / librccl first)

import chiara_amd  # noqa: E402,F401  (loads libchiara.so against them)


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libcoresidency_probe.so"))
    args = [b"coresidency_probe"] + [a.encode() for a in sys.argv[1:]]
    argv = (ctypes.c_char_p * len(args))(*args)
    lib.probe_main.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
    sys.stdout.flush()
    rc = lib.probe_main(len(args), argv)
    sys.exit(rc)


if __name__ == "__main__":
    main()
