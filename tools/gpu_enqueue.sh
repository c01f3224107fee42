#!/bin/bash
# Tree kernel f32+bf16 microbench, and the N>1 line's host-enqueue cost at 8 slices (ranks share
# the one GPU over RCCL's socket transport: only the host-side numbers mean anything).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 300 python tools/tree_bench.py > $OUT/tree_bench2.json 2> $OUT/tree_bench2.err; rc=$?
echo "tree_bench rc=$rc"; cat $OUT/tree_bench2.json; [ $rc -eq 0 ] || { tail -20 $OUT/tree_bench2.err; exit $rc; }
for N in 4 8; do
  CHR_SLICES=8 CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2981$N bench.py --gpus $N --steps 10 --warmup 2 --count $((1<<20)) --no-compare > $OUT/bench_enq_n$N.json 2> $OUT/bench_enq_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; cat $OUT/bench_enq_n$N.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_enq_n$N.err; exit $rc; }
done
echo ALL_DONE
