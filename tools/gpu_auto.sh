#!/bin/bash
# CHR_SCHEDULE_AUTO: its RCCL test (4 ranks on the one GPU, socket transport), then the N>1 bench
# line with the metric on AUTO at N=2 and N=8 (GB/s meaningless on one GPU; the tuned choice and
# every field must be produced).  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_rccl_multirank.py -k "auto or schedules_and_overlap" > $OUT/pytest_auto.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/pytest_auto.log; [ $rc -eq 0 ] || exit $rc
for N in 2 8; do
  CHR_TUNE_VERBOSE=1 CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2999$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<21)) > $OUT/bench_auto_n$N.json 2> $OUT/bench_auto_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_auto_n$N.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_auto_n$N.json'));print(d['config']['schedule'], sorted(d['compare']))"
  grep "\[chiara\] tune" $OUT/bench_auto_n$N.err | head -20
done
echo ALL_DONE
