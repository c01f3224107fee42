#!/bin/bash
# Occupancy-cap sweep of the co-residency probe: per cap in $CAPS, the admission of an RCCL-sized
# kernel (19 744 / 37 664 B LDS) next to a 64 MiB-piece tree launch and the C4 slice, plus the
# residency census.  gpurun -- bash tools/gpu_cores_sweep.sh  (TAG, CAPS from the environment)
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${TAG:-cores5}; mkdir -p $O
P=tools/coresidency_probe
timeout -k 10 60 $P --census 1 > $O/census.jsonl 2>&1 || exit 1
cat $O/census.jsonl
r() { local n=$1; shift; timeout -k 10 60 "$@" > $O/$n.jsonl 2> $O/$n.err; local rc=$?; echo "== $n rc=$rc"; grep -o '"tree_alone_frac.*' $O/$n.jsonl; [ $rc -eq 0 ] || exit $rc; }
for cap in ${CAPS:-10 11 12 13 14 16}; do
  for lds in 19744 37664; do
    r cap${cap}_lds${lds}_p64 env CHR_WG_PER_CU_TREE=$cap $P --mode mimic --reps 3 --piece 64 --launches 1 --xfer 16 --mimic-lds $lds
  done
  r cap${cap}_c4 env CHR_WG_PER_CU_TREE=$cap $P --mode mimic --reps 3
done
echo DONE
