#!/bin/bash
# Round 2, GPU call A: the new parity / hardening tests, then the C2 bench at the driver's settings.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rccl_multirank.py::test_rccl_graph_cache_survives_scratch_growth_world4 \
  tests/test_gpu_rccl_multirank.py::test_rccl_lost_peer_times_out_world4 \
  "tests/test_gpu_collectives.py::test_c4_c5_full_size_bit_exact_vs_oracle" \
  tests/test_gpu_collectives.py::test_c3_full_size_windowed_inputs_from_device \
  tests/test_gpu_ref_harness.py::test_own_harnesses_device_resident \
  > gpurun_out/pytest_a.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_w5.json 2> gpurun_out/bench_s20_w5.err && \
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_s200.json 2> gpurun_out/bench_s200.err
