#!/bin/bash
# Fused-tree kernel: its GPU tests, the collective goldens (flat plans now use it), and the
# tree-vs-folds microbench.  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_collectives.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_tree.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_tree.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tree_bench.py > $OUT/tree_bench.json 2> $OUT/tree_bench.err; rc=$?
echo "tree_bench rc=$rc"; cat $OUT/tree_bench.json; [ $rc -eq 0 ] || { tail -20 $OUT/tree_bench.err; exit $rc; }
echo ALL_DONE
