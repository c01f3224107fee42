#!/bin/bash
# Round 2, GPU call C: the whole -m gpu suite (as the driver runs it), smoke, then the C2 bench and
# its rocprofv3 kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/ \
  > gpurun_out/pytest_full.txt 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
