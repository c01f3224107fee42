#!/bin/bash
# Round-end re-check: every GPU test, smoke(), the N=1 bench line, and the N>1 line at N=2 and N=8
# with every compare entry (ranks sharing the one GPU over RCCL's socket transport).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
for N in 2 8; do
  CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2999$N bench.py --gpus $N --steps 3 --warmup 1 --count $((1<<21)) > $OUT/bench_all_n$N.json 2> $OUT/bench_all_n$N.err; rc=$?
  echo "bench N=$N rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_all_n$N.err; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/bench_all_n$N.json'));print(d['config']['schedule'], sorted(d['compare']), d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
echo ALL_DONE
