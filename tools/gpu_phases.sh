#!/bin/bash
# Per-phase transfer timing (profile_phases) in the N>1 line + RCCL multirank tests.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl_multirank.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest_rccl.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_rccl.log; [ $rc -eq 0 ] || exit $rc
for N in 4; do
  CHR_SLICES=4 CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2995$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<22)) --no-compare --no-cpu-baseline > $OUT/bench_ph_n$N.json 2> $OUT/bench_ph_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench_ph_n$N.json'));print(d['ms_per_step'], d['phase_transfer_ms'], d['roofline']['kernel_ms_per_call'])"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_ph_n$N.err; exit $rc; }
done
echo ALL_DONE
