#!/bin/bash
# tools/dtype_bench.py with tools/ab_old/libchiara.so (a build of an earlier commit) against the in-tree build,
# alternating, 2 rounds; the builds are swapped in place on the box's scratch copy.   gpurun -- bash tools/gpu_dtype_ab.sh
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-dtype_ab}; mkdir -p $O
LIB=configurable-hierarchical-allreduce-algorithms_amd/chiara_amd/libchiara.so
[ -f tools/ab_old/libchiara.so ] || { echo "no tools/ab_old/libchiara.so"; exit 2; }
mkdir -p /tmp/ab_new && cp $LIB /tmp/ab_new/libchiara.so
for rd in 1 2; do
  for b in old new; do
    if [ $b = old ]; then cp tools/ab_old/libchiara.so $LIB; else cp /tmp/ab_new/libchiara.so $LIB; fi
    timeout -k 10 240 python3 tools/dtype_bench.py --label ${b}_r$rd >> $O/dtype_ab.jsonl 2>> $O/dtype_ab.err \
      || { echo "$b r$rd failed"; cp /tmp/ab_new/libchiara.so $LIB; exit 1; }
    echo "== $b r$rd done"
  done
done
cp /tmp/ab_new/libchiara.so $LIB
echo DONE
