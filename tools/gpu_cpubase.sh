#!/bin/bash
# N>1 line with the reference CPU+MPI baseline (ranks share the one GPU: GPU numbers meaningless).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
for N in 2 4 8; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2991$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<22)) --no-compare > $OUT/bench_cpu_n$N.json 2> $OUT/bench_cpu_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench_cpu_n$N.json'));print(d['value'], d['cpu_baseline'])"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_cpu_n$N.err; exit $rc; }
done
echo ALL_DONE
