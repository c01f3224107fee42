# Round-6 HEAD context records: C2 over 200 steps, the sweep, the host-memory (e2e) rate, and the N = 4 line at
# 1 GiB per rank with virtual hosts (its fold's PMC binding and result check)
set -u -o pipefail
bash tools/gpu.sh bench200 sweep e2e || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
CHR_BENCH_VIRTUAL_HOSTS=1 CHR_SCHEDULE=flat CHR_BENCH_DEADLINE_S=200 timeout -k 10 600 python bench.py --gpus 4 \
  --count 268435456 > gpurun_out/bench_launch_n4_1gib_flat.json 2> gpurun_out/bench_launch_n4_1gib_flat.err || exit $?
echo done
