#!/bin/bash
# Round 2, GPU call E: counter list, the m-stream layout probe, full-size C4/C5 parity at both
# pipeline depths (LocalGroup and RCCL), and the 8-rank bench rehearsal at 1 GiB per rank.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
timeout -k 10 400 python tools/mstream_probe.py > gpurun_out/mstream_probe.jsonl 2> gpurun_out/mstream_probe.err && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  tests/test_gpu_collectives.py::test_c4_c5_full_size_bit_exact_vs_oracle \
  tests/test_gpu_rccl_multirank.py::test_rccl_c4_c5_full_size_bit_exact_world8 \
  > gpurun_out/pytest_e.txt 2>&1 && \
CHR_BENCH_VIRTUAL_HOSTS=1 CHR_SCHEDULE=flat timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29618 bench.py --gpus 8 --steps 2 --warmup 1 \
  --no-compare > gpurun_out/bench_n8_rehearsal_1gib.json 2> gpurun_out/bench_n8_rehearsal_1gib.err
