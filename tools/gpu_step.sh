#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export TESTS="tests/test_gpu_ref_harness.py" TAG=ref_harness TEST_LIMIT=400
bash tools/gpu.sh tests smoke bench pmc prof kernels treepmc || exit 1
