#!/bin/bash
# A/B of the vector kernels' workgroup size (CHR_REDUCE_BLOCK = 256 vs 64) and the first-slot
# accumulator policy (CHR_REDUCE_ACC0) through the product API: the C2 bench line (3 alternating
# rounds), then the size sweep and the tree-vs-folds bench per setting.
# Each GPU step has its own time limit; a failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
CFGS=${CFGS:-"256:d 64:d 256:1 64:1"}
for r in 1 2 3; do
  for c in $CFGS; do
    bl=${c%%:*}; a=${c##*:}; [ "$a" = d ] && unset CHR_REDUCE_ACC0 || export CHR_REDUCE_ACC0=$a
    CHR_REDUCE_BLOCK=$bl timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > $OUT/bench_b${bl}_a${a}_r$r.json 2>/dev/null; rc=$?
    [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('$OUT/bench_b${bl}_a${a}_r$r.json'));print('block $bl acc0 $a round $r', d['value'], d['roofline']['frac'])"
  done
done
if [ "${SWEEP:-1}" = 1 ]; then
  for c in $CFGS; do
    bl=${c%%:*}; a=${c##*:}; [ "$a" = d ] && unset CHR_REDUCE_ACC0 || export CHR_REDUCE_ACC0=$a
    CHR_REDUCE_BLOCK=$bl timeout -k 10 300 python bench.py --sweep --steps 20 --warmup 5 --no-cpu-baseline > $OUT/sweep_b${bl}_a$a.json 2> $OUT/sweep_b${bl}_a$a.err; rc=$?
    [ $rc -eq 0 ] || { echo "sweep rc=$rc"; exit $rc; }
    CHR_REDUCE_BLOCK=$bl timeout -k 10 300 python tools/tree_bench.py > $OUT/tree_b${bl}_a$a.json 2> $OUT/tree_b${bl}_a$a.err; rc=$?
    [ $rc -eq 0 ] || { echo "tree rc=$rc"; exit $rc; }
  done
fi
echo ALL_DONE
