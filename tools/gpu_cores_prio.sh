#!/bin/bash
# Can a high-priority transfer stream let RCCL's kernel in beside trees at the standalone cap 16?  The in-collective
# cap of 12 exists only so that rcclGenericKernel (256 threads, ~288 VGPRs per wave, 20-37 KiB LDS) finds room while a
# tree launch streams (profiles/r03/coresidency/); it costs the trees 2-9 %.  If the dispatcher admits
# a high-priority queue's workgroup first when a tree workgroup retires, cap 16 with the transfers on a priority
# stream keeps both.  Mimic kernel at both LDS sizes beside the 64 MiB-piece launch and the C4 slice, and the real
# RCCL kernel under rocprofv3; caps 16 and 12, prio 0 / 1, 2 rounds.   gpurun -- bash tools/gpu_cores_prio.sh
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-cores_prio}; mkdir -p $O
P=tools/coresidency_probe
r() { local n=$1; shift; timeout -k 10 90 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"
      grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for rd in 1 2; do
  for cap in 16 12; do
    for pr in 0 1; do
      for lds in 19744 37664; do
        r c${cap}_p${pr}_lds${lds}_p64_r$rd env CHR_WG_PER_CU_TREE=$cap $P --mode mimic --prio $pr --reps 3 --piece 64 \
          --launches 1 --xfer 16 --mimic-lds $lds
      done
      r c${cap}_p${pr}_c4_r$rd env CHR_WG_PER_CU_TREE=$cap $P --mode mimic --prio $pr --reps 3
      d=$O/c${cap}_p${pr}_rccl_r$rd
      CHR_WG_PER_CU_TREE=$cap timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run \
        -- $P --mode rccl --prio $pr --reps 3 > $d.jsonl 2> $d.err || exit 1
      python3 tools/coresidency_report.py $d/run_kernel_trace.csv c${cap}_p${pr}_rccl_r$rd >> $O/report.jsonl
      grep summary $O/report.jsonl | tail -1
    done
  done
done
echo DONE
