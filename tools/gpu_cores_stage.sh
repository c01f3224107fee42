#!/bin/bash
# Co-residency of an RCCL-sized kernel beside the in-collective trees, one-vector trip vs the LDS-staged shape
# (CHR_TREE_STAGE=0 / 1; reduce_tree.hpp k_reduce_tree_staged, 56-64 VGPRs): the register-held U = 2 shape locked
# RCCL's waves out (profiles/r05/cores_u/); the staged one must not.  Cap 12, mimic kernel at torch's and ROCm's RCCL
# LDS beside the 64 MiB-piece launch and the C4 slice, then the real RCCL kernel (--mode rccl) under rocprofv3,
# alternating, 2 rounds.  gpurun -- bash tools/gpu_cores_stage.sh
# CHR_TREE_STAGE existed in a round-5 working tree only (the staged shape also cost RCCL: profiles/r05/cores_stage/).
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-cores_stage}; mkdir -p $O
P=tools/coresidency_probe
r() { local n=$1; shift; timeout -k 10 90 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"
      grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for rd in 1 2; do
  for u in 0 1; do
    for lds in 19744 37664; do
      r u${u}_lds${lds}_p64_r$rd env CHR_WG_PER_CU_TREE=12 CHR_TREE_STAGE=$u $P --mode mimic --reps 3 --piece 64 --launches 1 \
        --xfer 16 --mimic-lds $lds
    done
    r u${u}_c4_r$rd env CHR_WG_PER_CU_TREE=12 CHR_TREE_STAGE=$u $P --mode mimic --reps 3
    d=$O/u${u}_rccl_r$rd
    CHR_WG_PER_CU_TREE=12 CHR_TREE_STAGE=$u timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run \
      -- $P --mode rccl --reps 3 > $d.jsonl 2> $d.err || exit 1
    python3 tools/coresidency_report.py $d/run_kernel_trace.csv u${u}_rccl_r$rd >> $O/report.jsonl
    grep summary $O/report.jsonl | tail -1
  done
done
echo DONE
