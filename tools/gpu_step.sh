#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 tools/reduce_microbench focus21 > gpurun_out/focus21.txt 2>&1 || exit 1
N=4 bash tools/gpu.sh rehearse || exit 1
