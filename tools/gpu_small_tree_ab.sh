#!/bin/bash
# Shape A/B of the N = 4 / N = 2 lines' 4- and 2-leaf streaming trees (tools/small_tree_ab.py), alternating
# variants, 2 rounds:  policy | runs 256 KiB + cap 12 | runs 256 KiB + cap 16 | cap 12 (the in-collective cap).
#   gpurun -- bash tools/gpu_small_tree_ab.sh
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${TAG:-small_tree_ab}; mkdir -p $O
for rd in 1 2; do
  for v in policy r256c12 r256c16 c12 r256; do
    case $v in
      policy) E="" ;;
      r256c12) E="CHR_XCD_RUN_KIB=256 CHR_WG_PER_CU_TREE=12" ;;
      r256c16) E="CHR_XCD_RUN_KIB=256 CHR_WG_PER_CU_TREE=16" ;;
      c12) E="CHR_WG_PER_CU_TREE=12" ;;
      r256) E="CHR_XCD_RUN_KIB=256" ;;
    esac
    env $E timeout -k 10 180 python3 tools/small_tree_ab.py --label ${v}_r$rd >> $O/small_tree_ab.jsonl \
      2>> $O/small_tree_ab.err || { echo "$v r$rd failed"; exit 1; }
    echo "== $v r$rd done"
  done
done
echo DONE
