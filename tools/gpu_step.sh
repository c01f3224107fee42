#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/cks
ck() {  # ck <tag> [ENV=VAL ...]: the small-geometry in-collective rows under the given knobs
  local tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --collective-kernels-small > gpurun_out/cks/$tag.json 2> gpurun_out/cks/$tag.err || exit 1
  echo "[$(date +%T)] $tag done"
}
for r in 1 2; do
  ck default_r$r
  ck cap12_runs256_r$r CHR_WG_PER_CU_TREE=12 CHR_XCD_RUN_KIB=256
  ck cap12_r$r CHR_WG_PER_CU_TREE=12
  ck cap16_r$r CHR_WG_PER_CU_TREE=16
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/ck_prof" -o run -- python3 bench.py --collective-kernels > gpurun_out/ck_prof.json 2> gpurun_out/ck_prof.err || exit 1
echo ALL_DONE
