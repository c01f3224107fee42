#!/bin/bash
# N>1 bench line rehearsal with the full compare block and the CPU baseline (ranks share the one
# GPU over RCCL's socket transport: GB/s meaningless; every field must be produced without error).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
for N in 2 8; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2999$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<21)) > $OUT/bench_all_n$N.json 2> $OUT/bench_all_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; python -c "import json;d=json.load(open('$OUT/bench_all_n$N.json'));print(sorted(d['compare']), d['phase_transfer_ms'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_all_n$N.err; exit $rc; }
done
echo ALL_DONE
