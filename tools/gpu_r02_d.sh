#!/bin/bash
# Round 2, GPU call D: batched trees (kernel, goldens, full-size C4), the shim type table, the tree
# micro-benchmark (separate vs batched, cold vs warm leaves), and the C2 bench under rocprofv3.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu \
  tests/test_gpu_tree.py tests/test_gpu_ref_harness.py \
  tests/test_gpu_collectives.py::test_local_group_matches_reference_golden \
  tests/test_gpu_collectives.py::test_integer_types_and_logical_bitwise_ops_match_reference_golden \
  "tests/test_gpu_collectives.py::test_c4_c5_full_size_bit_exact_vs_oracle[f32-flat]" \
  "tests/test_gpu_collectives.py::test_baseline_geometries_vs_oracle" \
  > gpurun_out/pytest_d.txt 2>&1 && \
timeout -k 10 300 python tools/tree_bench.py > gpurun_out/tree_bench.json 2> gpurun_out/tree_bench.err && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
