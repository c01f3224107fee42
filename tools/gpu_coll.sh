#!/bin/bash
# Collective-level GPU tests (LocalGroup goldens, every schedule, RCCL multi-rank incl. phase profiling).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_collectives.py tests/test_gpu_rccl_multirank.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest_coll.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_coll.log; [ $rc -eq 0 ] || exit $rc
echo ALL_DONE
