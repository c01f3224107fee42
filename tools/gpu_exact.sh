#!/bin/bash
# Exact schedule on the device (LocalGroup goldens, RCCL multi-rank) + N>1 bench rehearsal
# (ranks share the one GPU over RCCL's socket transport: GB/s meaningless, the line's fields are the point).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_rccl_multirank.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest_exact.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_exact.log; [ $rc -eq 0 ] || exit $rc
for N in 2 4; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2971$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<22)) > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; cat $OUT/bench_n$N.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_n$N.err; exit $rc; }
done
echo ALL_DONE
