#!/bin/bash
# Co-residency of an RCCL-sized kernel beside the in-collective trees, U = 1 vs U = 2 (reduce_tree.hpp
# tree_u_wide): the U = 2 shape needs 82-90 VGPRs per wave against U = 1's 50-58, and rcclGenericKernel needs a
# wave slot with ~288 VGPRs free on each SIMD of a CU.  At the in-collective cap 12 (CHR_WG_PER_CU_TREE=12),
# mimic kernel at torch's and ROCm's RCCL LDS, the 64 MiB-piece launch and the C4 slice, then the real RCCL
# kernel (--mode rccl) under rocprofv3, alternating U, 2 rounds.  gpurun -- bash tools/gpu_cores_u.sh
# CHR_TREE_U exists at commit bace861 only (U = 2 lost RCCL its co-residency: profiles/r05/cores_u/).
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-cores_u}; mkdir -p $O
P=tools/coresidency_probe
r() { local n=$1; shift; timeout -k 10 90 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"
      grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for rd in 1 2; do
  for u in 1 2; do
    for lds in 19744 37664; do
      r u${u}_lds${lds}_p64_r$rd env CHR_WG_PER_CU_TREE=12 CHR_TREE_U=$u $P --mode mimic --reps 3 --piece 64 --launches 1 \
        --xfer 16 --mimic-lds $lds
    done
    r u${u}_c4_r$rd env CHR_WG_PER_CU_TREE=12 CHR_TREE_U=$u $P --mode mimic --reps 3
    d=$O/u${u}_rccl_r$rd
    CHR_WG_PER_CU_TREE=12 CHR_TREE_U=$u timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run \
      -- $P --mode rccl --reps 3 > $d.jsonl 2> $d.err || exit 1
    python3 tools/coresidency_report.py $d/run_kernel_trace.csv u${u}_rccl_r$rd >> $O/report.jsonl
    grep summary $O/report.jsonl | tail -1
  done
done
echo DONE
