# The N = 4 line at 1 GiB per rank with virtual hosts (flat): its fold's PMC binding and result check.  A heartbeat
# file keeps the call visibly alive while the socket-bound steps run (bench.py prints its line only at the end).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/heartbeat_n4.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
CHR_BENCH_VIRTUAL_HOSTS=1 CHR_SCHEDULE=flat CHR_BENCH_DEADLINE_S=200 timeout -k 10 600 python bench.py --gpus 4 \
  --count 268435456 > gpurun_out/bench_launch_n4_1gib_flat.json 2> gpurun_out/bench_launch_n4_1gib_flat.err || exit $?
echo done
