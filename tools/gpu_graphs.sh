#!/bin/bash
# Graph replay of collectives: its RCCL test (4 ranks on the one GPU), then the N>1 line at N=4 with
# the small-message block (eager vs graph; socket transport, so only the host share is meaningful).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_rccl_multirank.py -k "graph or auto" > $OUT/pytest_graphs.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/pytest_graphs.log; [ $rc -eq 0 ] || exit $rc
CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29994 bench.py --gpus 4 --steps 3 --warmup 1 --count $((1<<20)) --no-cpu-baseline > $OUT/bench_graphs_n4.json 2> $OUT/bench_graphs_n4.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_graphs_n4.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_graphs_n4.json'));print(d['config']['schedule'], d['compare']['small_messages'])"
echo ALL_DONE
