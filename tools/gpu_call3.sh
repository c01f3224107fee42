# The N = 2 launcher line (rccl library / version), the whole -m gpu suite (child-process tests first, 420 s budget
# strict), then C4 / C5 rank 0's own 8-leaf grids at the in-collective cap with the tree ACC0 slot off / on alternating
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/c3; mkdir -p $O
CHR_BENCH_VIRTUAL_HOSTS=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_launch_n2.json 2> $O/bench_launch_n2.err || exit $?
CHR_GPU_SUITE_BUDGET_STRICT=1 timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread --durations=0 -m gpu tests/ > $O/pytest_suite.txt 2> $O/pytest_suite.err
rc=$?; echo "suite rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
for r in 1 2; do
  CHR_WG_PER_CU_TREE=12 timeout -k 10 300 python bench.py --rank-trees > $O/rt8_off_$r.json 2> $O/rt8_off_$r.err || exit $?
  CHR_TREE_ACC0=1 CHR_WG_PER_CU_TREE=12 timeout -k 10 300 python bench.py --rank-trees > $O/rt8_acc0_$r.json 2> $O/rt8_acc0_$r.err || exit $?
done
echo done
