#!/bin/bash
# Kernel-policy check: kernel tests, the C2 bench line, the size sweep, the per-slot microbench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q > $OUT/pytest_kernels.log 2>&1; rc=$?; echo "kernel tests rc=$rc"; tail -2 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sweep > $OUT/bench_sweep.json 2> $OUT/bench_sweep.err; rc=$?
echo "sweep rc=$rc"; grep sweep $OUT/bench_sweep.err | grep -E "bucket= *(67108864|268435456|1073741824)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 ./tools/reduce_microbench focus4 > $OUT/microbench_focus4.txt 2>&1; rc=$?; echo "focus4 rc=$rc"; grep -E "all-nt U4|acc0 dflt U4|libchiara" $OUT/microbench_focus4.txt
echo ALL_DONE
