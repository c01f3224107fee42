#!/bin/bash
# One GPU-box session: GPU tests, a bench line, a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out
STEPS=${STEPS:-200}
echo "host: nproc=$(nproc) mpi=$(ls /opt/conda/bin/mpiexec 2>/dev/null)" > $OUT/env.txt
rocm-smi --showproductname >> $OUT/env.txt 2>&1 || true
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU step failed rc=$rc, stopping"; exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --maxfail=30 ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log; ok $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 300 python bench.py --steps $STEPS --warmup 20 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
  echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
     python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err; rc=$?
  echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find $OUT/prof -name "*stats*" | head
fi
if [ "${PMC:-0}" = "1" ]; then
  export TMPDIR=/tmp
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_$ctr -o run -- \
       python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err; rc=$?
    echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
echo ALL_DONE
