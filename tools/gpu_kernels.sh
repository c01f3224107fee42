#!/bin/bash
# Kernel-level GPU tests (fold + tree kernels, bit-exact vs the oracle) and the tree microbench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_kernels.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tree_bench.py > $OUT/tree_bench3.json 2> $OUT/tree_bench3.err; rc=$?
echo "tree_bench rc=$rc"; cat $OUT/tree_bench3.json; [ $rc -eq 0 ] || { tail -20 $OUT/tree_bench3.err; exit $rc; }
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sweep > $OUT/bench_sweep3.json 2> $OUT/bench_sweep3.err; rc=$?
echo "sweep rc=$rc"; grep "sweep bf16\|sweep f32 m=1" $OUT/bench_sweep3.err | tail -30
echo ALL_DONE
