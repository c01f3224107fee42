#!/bin/bash
# Ad-hoc GPU step list for one gpurun call (edited per call; tools/gpu.sh holds the steps).
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ab_dual; mkdir -p $O
for r in 1 2; do
  for d in 0 1; do
    CHR_DUAL_COMPUTE=$d timeout -k 10 300 python bench.py --collective-kernels > $O/ck_dual${d}_r$r.json 2> $O/ck_dual${d}_r$r.err || exit 1
    echo "dual=$d r=$r $(python -c "import json;d=json.load(open('$O/ck_dual${d}_r$r.json'))['collective_kernels']['rows'];print({k: v['frac'] for k, v in d.items() if 'alone' not in k})")"
  done
done
