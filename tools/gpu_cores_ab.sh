#!/bin/bash
# A/B of two builds of libchiara.so beside RCCL, alternating, 2 rounds: A = tools/ab_old/libchiara.so (a build of
# an earlier commit, made by hand), B = the in-tree build.  Per round and build, at the in-collective cap 12:
#   * the co-residency check of tools/gpu_cores_check.sh on DT's trees (the mimic at torch's and ROCm's RCCL LDS
#     beside the 64 MiB-piece launch and the C4/C5 slice; the real RCCL kernel under rocprofv3);
#   * the same trees at the stand-alone policy cap (tree_alone_frac of the 64 MiB-piece launch);
#   * with LEAVES=8 (C4 / C5's trees), one GPU's own C4 / C5 grids (bench.py --rank-trees under rocprofv3).
# The probe picks the build by LD_LIBRARY_PATH (its RUNPATH comes after it); bench.py loads the in-tree file, so
# the builds are swapped in place on the box's scratch copy.
#   gpurun -- bash tools/gpu_cores_ab.sh          (DT=bf16|f32, LEAVES=8|4|2, TAG names the output directory)
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-cores_ab}; mkdir -p $O
P=tools/coresidency_probe
LIB=configurable-hierarchical-allreduce-algorithms_amd/chiara_amd/libchiara.so
DT=${DT:-bf16}
LEAVES=${LEAVES:-8}
A="--dtype $DT --leaves $LEAVES"
[ -f tools/ab_old/libchiara.so ] || { echo "no tools/ab_old/libchiara.so"; exit 2; }
mkdir -p /tmp/ab_new && cp $LIB /tmp/ab_new/libchiara.so
r() { local n=$1; shift; timeout -k 10 90 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"
      grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for rd in 1 2; do
  for b in old new; do
    if [ $b = old ]; then D=$PWD/tools/ab_old; else D=/tmp/ab_new; fi
    cp $D/libchiara.so $LIB
    for lds in 19744 37664; do
      r ${b}_lds${lds}_p64_r$rd env LD_LIBRARY_PATH=$D CHR_WG_PER_CU_TREE=12 $P --mode mimic --reps 3 --piece 64 \
        --launches 1 --xfer 16 --mimic-lds $lds $A
    done
    r ${b}_slice_r$rd env LD_LIBRARY_PATH=$D CHR_WG_PER_CU_TREE=12 $P --mode mimic --reps 3 $A
    r ${b}_policy_p64_r$rd env LD_LIBRARY_PATH=$D $P --mode mimic --reps 3 --piece 64 --launches 1 --xfer 16 $A
    d=$O/${b}_rccl_r$rd
    LD_LIBRARY_PATH=$D CHR_WG_PER_CU_TREE=12 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
      -d $PWD/$d -o run -- $P --mode rccl --reps 3 $A > $d.jsonl 2> $d.err || exit 1
    python3 tools/coresidency_report.py $d/run_kernel_trace.csv ${b}_rccl_r$rd >> $O/report.jsonl
    grep summary $O/report.jsonl | tail -1
    [ "$LEAVES" = 8 ] || continue
    d=$O/${b}_ranktrees_r$rd
    CHR_WG_PER_CU_TREE=12 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run \
      -- python3 bench.py --rank-trees > $d.json 2> $d.err || exit 1
    python3 tools/rank_trees_summary.py $d.json $d > $d.summary.json || exit 1
    echo "== ${b}_ranktrees_r$rd done"
  done
done
cp /tmp/ab_new/libchiara.so $LIB
echo DONE
