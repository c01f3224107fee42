#!/bin/bash
# A/B through the product API: C2 (bench.py, 200 steps) with the policy XCD map vs 256 KiB runs
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab_runs
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2 3; do
  for v in policy 256; do
    if [ "$v" = policy ]; then unset CHR_XCD_RUN_KIB; else export CHR_XCD_RUN_KIB=$v; fi
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_runs/c2_${v}_r${r}.json 2>/dev/null || exit 1
    echo "c2 runs=$v r=$r $(python -c "import json;d=json.load(open('gpurun_out/ab_runs/c2_${v}_r${r}.json'));print(d['value'], d['roofline']['frac'])")"
  done
done
unset CHR_XCD_RUN_KIB
echo AB_DONE
