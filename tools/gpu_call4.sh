# Tree ACC0 slot off / on, by rocprof kernel duration: one GPU's own C4 / C5 grids at the in-collective cap (bench.py
# --rank-trees under rocprofv3 --kernel-trace), and the 8-leaf tree alone (tools/tree_pmc.py), 2 alternating rounds
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/c4; mkdir -p $O
for r in 1 2; do
  for v in off acc0; do
    a=$([ $v = acc0 ] && echo 1 || echo 0)
    CHR_TREE_ACC0=$a CHR_WG_PER_CU_TREE=12 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$O/rt_${v}_$r" -o run -- python3 bench.py --rank-trees > $O/rt_${v}_$r.json 2> $O/rt_${v}_$r.err || exit $?
    CHR_TREE_ACC0=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$O/tree_${v}_$r" -o run -- python3 tools/tree_pmc.py 40 > $O/tree_${v}_$r.txt 2>&1 || exit $?
  done
done
echo done
