#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
export TESTS="tests/test_gpu_collectives.py" TAG=collectives TEST_LIMIT=600
bash tools/gpu.sh tests kernels || exit 1
