#!/bin/bash
# Round 2, GPU call G: big-stagger layouts for the m=3/m=7 1 GiB drop, and the collective's own
# fused reductions at C4/C5 full size (8 virtual ranks, HIP events).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python tools/mstream_probe.py --ms 3,7 --mib 512,1024 \
  --layouts sep,slab,slab+64m,slab+96m4k,slab+192m,slab+320m > gpurun_out/mstream_probe2.jsonl 2> gpurun_out/mstream_probe2.err && \
timeout -k 10 400 python bench.py --collective-kernels > gpurun_out/collective_kernels.json 2> gpurun_out/collective_kernels.err
