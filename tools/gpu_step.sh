#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
LIB=configurable-hierarchical-allreduce-algorithms_amd/chiara_amd/libchiara.so
# 1. the exhaustive scalar-path tree test against the library before the slot fix (expected to fail)
cp $LIB /tmp/libchiara_new.so && cp tools/ab_lib/libchiara_before_slot_fix.so $LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_tree.py -k "every_program" > gpurun_out/pytest_tree_before_fix.txt 2>&1
echo "before-fix rc=$?" >> gpurun_out/pytest_tree_before_fix.txt
cp /tmp/libchiara_new.so $LIB
# 2. with the fix: tree, collectives (one-shot goldens), RCCL schedules + AUTO
export TESTS="tests/test_gpu_tree.py tests/test_gpu_collectives.py tests/test_gpu_rccl_multirank.py::test_rccl_schedules_and_overlap_world4 tests/test_gpu_rccl_multirank.py::test_rccl_auto_schedule_world4" TAG=fix TEST_LIMIT=800
bash tools/gpu.sh tests treepmc || exit 1
