#!/bin/bash
# new GPU tests + size sweep + N>1 bench rehearsal on one GPU
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_ref_harness.py tests/test_gpu_rccl_multirank.py -q > $OUT/pytest_extra.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_extra.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sweep > $OUT/bench_sweep.json 2> $OUT/bench_sweep.err; rc=$?
echo "sweep rc=$rc"; tail -40 $OUT/bench_sweep.err; [ $rc -eq 0 ] || exit $rc
for N in 2 4; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<22)) > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; cat $OUT/bench_n$N.json; tail -3 $OUT/bench_n$N.err; [ $rc -eq 0 ] || exit $rc
done
echo ALL_DONE
