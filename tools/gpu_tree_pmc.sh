#!/bin/bash
# HBM traffic of the fused tree kernel: separate --pmc passes (FETCH_SIZE, WRITE_SIZE) + kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tpmc_$ctr -o run -- python3 $GRAFT_REPO_ROOT/tools/tree_pmc.py 40 > $OUT/tpmc_$ctr.log 2>&1; rc=$?
  echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/tpmc_$ctr.log; exit $rc; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tprof -o run -- python3 $GRAFT_REPO_ROOT/tools/tree_pmc.py 40 > $OUT/tprof.log 2>&1; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $OUT/tpmc_FETCH_SIZE $OUT/tpmc_WRITE_SIZE tree_f32_sum_8leaves_64MiB $((9*64*1024*1024)) - k_reduce_tree
cat $(find $OUT/tprof -name "*kernel_stats.csv")
echo ALL_DONE
