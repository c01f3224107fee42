#!/bin/bash
# One script for every GPU-box session (replaces the per-call tools/gpu_*.sh of rounds 1-2).
#
#   gpurun --timeout 1200 -- bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in the order given; each GPU step has its own time limit and the first failure
# (test failure, fault, abort, time limit) ends the script, so nothing more touches the GPU.
#   suite      the whole -m gpu suite, as the driver runs it    -> pytest_suite.txt
#   tests      the pytest node ids in $TESTS                     -> pytest_${TAG:-tests}.txt
#   smoke      __graft_entry__.smoke()                           -> smoke.txt
#   bench      bench.py at the driver's settings (20 / 5)        -> bench.json
#   bench200   bench.py --steps 200 --warmup 20                  -> bench200.json
#   prof       rocprofv3 kernel trace + stats of the bench (csv) -> prof/
#   pmc        FETCH_SIZE and WRITE_SIZE passes of the bench     -> pmc_FETCH_SIZE/, pmc_WRITE_SIZE/
#   kernels    bench.py --collective-kernels (C4/C5 in-collective kernel rows) -> collective_kernels.json
#   ranktrees  bench.py --rank-trees, plain and under rocprofv3 --kernel-trace -> rank_trees.json, rank_trees_prof/
#   treepmc    rocprofv3 stats + FETCH_SIZE / WRITE_SIZE passes of the tree kernel alone (tools/tree_pmc.py)
#   treepmc42  the same for the 4- and 2-leaf trees (the tree API)
#   vecpmc     the same for the N = 2 / N = 4 lines' out-of-place folds (k_reduce_vec m = 1 at 128 MiB, m = 3 at 64 MiB)
#   e2e        bench.py --e2e: host-buffer (PCIe-inclusive) cost of the reference's contract -> e2e.json
#   sweep      bench.py --sweep: 1 KiB .. 1 GiB buckets, m = 1/3/7, fp32 + bf16 (table in sweep.json.err)
#   probe      tools/mstream_probe.py $PROBE_ARGS               -> mstream_probe.jsonl
#   tree       tools/tree_bench.py $TREE_ARGS                   -> tree_bench.json
#   launch     bench.py --gpus ${N:-2} with no external launcher (bench.py starts its own ranks;
#              virtual hosts: ranks share the one GPU, socket transport) -> bench_launch_n${N}.json
#   launch8    bench.py --gpus 8 at 1 GiB per rank, launcher + deadline, ranks sharing the GPU -> bench_launch_n8_1gib.json
#   rehearse   the N>1 bench line with ${N:-4} ranks sharing the one GPU (socket transport;
#              exercises the code path, its GB/s mean nothing)  -> bench_n${N}_rehearsal.json
# Everything lands under gpurun_out/.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout-method thread"

run() {  # run <seconds> <log> cmd...: the step's own limit; stop the script on failure
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$log" 2> "$OUT/$log.err"
  local rc=$?
  echo "[$(date +%T)] $log rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$log" "$OUT/$log.err"; exit $rc; fi
}

for step in "$@"; do
  case "$step" in
  suite) CHR_GPU_SUITE_BUDGET_STRICT=1 run 1100 pytest_suite.txt $PYT --timeout 900 --durations=0 -m gpu tests/ ;;
  tests) run "${TEST_LIMIT:-900}" "pytest_${TAG:-tests}.txt" python -u -m pytest -x -v --timeout-method thread --timeout 170 -m gpu ${TESTS:?set TESTS} ;;
  smoke) run 300 smoke.txt python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench) run 300 bench.json python bench.py --steps 20 --warmup 5 ;;
  bench200) run 300 bench200.json python bench.py --steps 200 --warmup 20 --no-cpu-baseline ;;
  prof) run 300 prof_bench.json rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run \
          -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline ;;
  pmc)
    for ctr in FETCH_SIZE WRITE_SIZE; do
      run 300 "pmc_$ctr.json" rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_$ctr" -o run \
        -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline
    done ;;
  kernels) run 400 collective_kernels.json python bench.py --collective-kernels ;;
  ranktrees)  # one GPU's own C4 / C5 grids: spans (JSON) and, under rocprofv3, each grid's kernel duration
    run 300 rank_trees.json python bench.py --rank-trees
    run 300 rank_trees_prof.json rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/rank_trees_prof" \
      -o run -- python3 bench.py --rank-trees ;;
  ranktrees12)  # the same grids at the in-collective cap: a multi-rank call runs its trees under CoresidentScope,
                # 12 workgroups per CU beside RCCL (reduce_common.hpp stream_wg_cap)
    CHR_WG_PER_CU_TREE=12 run 300 rank_trees_cap12_prof.json rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/rank_trees_cap12_prof" -o run -- python3 bench.py --rank-trees ;;
  treepmc)  # the fused tree alone at C4's shape (tools/tree_pmc.py): kernel stats, then FETCH / WRITE passes
    run 300 tree_prof.txt rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/tree_prof" -o run \
      -- python3 tools/tree_pmc.py 40
    for ctr in FETCH_SIZE WRITE_SIZE; do
      run 300 "tree_pmc_$ctr.txt" rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/tree_pmc_$ctr" -o run \
        -- python3 tools/tree_pmc.py 40
    done ;;
  vecpmc)  # the N = 2 / N = 4 lines' out-of-place folds -> vec{1,3}_prof/, vec{1,3}_pmc_*/
    for vm in 1 3; do
      vmib=$([ $vm = 1 ] && echo 128 || echo 64)
      run 300 "vec${vm}_prof.txt" rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/vec${vm}_prof" \
        -o run -- python3 tools/tree_pmc.py 40 --vec $vm --mib $vmib
      for ctr in FETCH_SIZE WRITE_SIZE; do
        run 300 "vec${vm}_pmc_$ctr.txt" rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/vec${vm}_pmc_$ctr" \
          -o run -- python3 tools/tree_pmc.py 40 --vec $vm --mib $vmib
      done
    done ;;
  treepmc42)  # the 4- and 2-leaf trees the same way -> tree{4,2}_prof/, tree{4,2}_pmc_*/
    for nl in 4 2; do
      run 300 "tree${nl}_prof.txt" rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/tree${nl}_prof" \
        -o run -- python3 tools/tree_pmc.py 40 --leaves $nl
      for ctr in FETCH_SIZE WRITE_SIZE; do
        run 300 "tree${nl}_pmc_$ctr.txt" rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/tree${nl}_pmc_$ctr" \
          -o run -- python3 tools/tree_pmc.py 40 --leaves $nl
      done
    done ;;
  sweep) run 600 sweep.json python bench.py --sweep --no-cpu-baseline ;;
  e2e) run 300 e2e.json python bench.py --e2e --no-cpu-baseline ;;
  probe) run 400 mstream_probe.jsonl python tools/mstream_probe.py ${PROBE_ARGS:-} ;;
  tree) run 400 tree_bench.json python tools/tree_bench.py ${TREE_ARGS:-} ;;
  launch)
    n=${N:-2}
    CHR_BENCH_VIRTUAL_HOSTS=1 CHR_BENCH_DEADLINE_S=${DEADLINE:-240} run 600 "bench_launch_n${n}.json" \
      python bench.py --gpus "$n" --steps 3 --warmup 1 --count $((1 << 21)) ;;
  launch8)  # the N=8 line at its real size (1 GiB per rank), 8 ranks sharing the one GPU over sockets: the
            # launcher and the deadline end to end (FLAT: AUTO's tuning over sockets would take minutes; a
            # heartbeat file keeps the call visibly alive while the socket-bound steps run)
    ( while sleep 50; do date +%T >> "$OUT/heartbeat_launch8.txt"; done ) &
    hb=$!
    trap 'kill $hb 2>/dev/null' EXIT
    CHR_BENCH_VIRTUAL_HOSTS=1 CHR_BENCH_DEADLINE_S=${DEADLINE:-150} CHR_SCHEDULE=${SCHED:-flat} run 700 "bench_launch_n8_1gib${SCHED:+_$SCHED}.json" \
      python bench.py --gpus 8 --steps 2 --warmup 1
    kill $hb ;;
  rehearse)
    n=${N:-4}
    CHR_BENCH_VIRTUAL_HOSTS=1 run 600 "bench_n${n}_rehearsal.json" python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29731 bench.py --gpus "$n" --steps 3 --warmup 1 \
      --count $((1 << 21)) ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_DONE
