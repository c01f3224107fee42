#!/bin/bash
# Round 2, GPU call B: kernel/tree suites (new integer types, refactored dispatch), the types
# goldens through the collectives, and C4/C5 at full size over RCCL (8 processes, socket transport).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_tree.py \
  "tests/test_gpu_collectives.py::test_integer_types_and_logical_bitwise_ops_match_reference_golden" \
  > gpurun_out/pytest_b1.txt 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rccl_multirank.py::test_rccl_c4_c5_full_size_bit_exact_world8 \
  > gpurun_out/pytest_b2.txt 2>&1
