#!/bin/bash
# Co-residency of an RCCL-sized kernel beside the shipped in-collective trees (cap 12): the mimic kernel at torch's
# and ROCm's RCCL LDS beside the 64 MiB-piece launch and the C4 slice, then the real RCCL kernel (--mode rccl) under
# rocprofv3, 2 rounds -- the check any change to the tree kernel's registers or workgroup lifetime must pass
# (profiles/r03/coresidency/: admitted within ~4-30 us, RCCL ~114-125 us beside the C4 slice).
# tests/test_kernel_resources.py holds the register half of it on every build (no GPU).
#   gpurun -- bash tools/gpu_cores_check.sh      (TAG names the output directory; DT=f32|bf16, LEAVES=8|4|2)
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-cores_check}; mkdir -p $O
P=tools/coresidency_probe
A="--dtype ${DT:-f32} --leaves ${LEAVES:-8}"
r() { local n=$1; shift; timeout -k 10 90 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"
      grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for rd in 1 2; do
  for lds in 19744 37664; do
    r lds${lds}_p64_r$rd env CHR_WG_PER_CU_TREE=12 $P --mode mimic --reps 3 --piece 64 --launches 1 --xfer 16 \
      --mimic-lds $lds $A
  done
  r c4_r$rd env CHR_WG_PER_CU_TREE=12 $P --mode mimic --reps 3 $A
  d=$O/rccl_r$rd
  CHR_WG_PER_CU_TREE=12 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run \
    -- $P --mode rccl --reps 3 $A > $d.jsonl 2> $d.err || exit 1
  python3 tools/coresidency_report.py $d/run_kernel_trace.csv rccl_r$rd >> $O/report.jsonl
  grep summary $O/report.jsonl | tail -1
done
echo DONE
