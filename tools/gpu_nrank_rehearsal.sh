#!/bin/bash
# N>1 bench rehearsal on the one-GPU box (socket transport between ranks sharing the GPU;
# the GB/s are meaningless, the point is that the line and its compare/roofline fields appear).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for N in 2 4; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2961$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<22)) > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; cat $OUT/bench_n$N.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_n$N.err; exit $rc; }
done
echo ALL_DONE
