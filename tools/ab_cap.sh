#!/bin/bash
# A/B of the occupancy cap through the product API (bench.py C2, mstream_probe m=3/7, collective kernels)
set -u -o pipefail
cd /root/repo
mkdir -p gpurun_out/cap
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2; do
  for c in 0 10 12 14 16; do
    CHR_WG_PER_CU_VEC=$c timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/cap/c2_cap${c}_r${r}.json 2>/dev/null || exit 1
    echo "c2 cap=$c r=$r $(python -c "import json;d=json.load(open('gpurun_out/cap/c2_cap${c}_r${r}.json'));print(d['value'], d['roofline']['frac'])")"
  done
done
for c in 0 12 10; do
  CHR_WG_PER_CU_VEC=$c timeout -k 10 300 python tools/mstream_probe.py --ms 3,7 --mib 256 --layouts sep --sets 1,8 > gpurun_out/cap/mstream_cap${c}.jsonl 2>/dev/null || exit 1
  echo "mstream cap=$c"; cat gpurun_out/cap/mstream_cap${c}.jsonl | cut -c1-300
done
for c in 0 8 10 12; do
  CHR_WG_PER_CU_TREE=$c timeout -k 10 400 python bench.py --collective-kernels > gpurun_out/cap/ck_tree_cap${c}.json 2>/dev/null || exit 1
  echo "tree cap=$c $(python -c "
import json;d=json.load(open('gpurun_out/cap/ck_tree_cap${c}.json'))['collective_kernels']['rows']
print({k:v['frac'] for k,v in d.items()})")"
done
echo AB_DONE
