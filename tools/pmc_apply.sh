#!/bin/bash
# Rebind profiles/pmc_latest.json to the PMC passes of one GPU session (tools/gpu.sh pmc treepmc vecpmc
# [treepmc42]), copied under DIR: each entry gets the kernel symbol and the source hash it was measured on
# (tools/pmc_provenance.py), which bench.py checks before it reports roofline.traffic.
#   bash tools/pmc_apply.sh profiles/r06/final
set -eu
D=${1:?directory holding the pmc_* / tree_pmc_* / vec*_pmc_* passes}
cd "$(dirname "$0")/.."
P="python3 tools/pmc_summary.py"
$P "$D/pmc_FETCH_SIZE" "$D/pmc_WRITE_SIZE" reduce_f32_sum_m1_64MiB 201326592 - k_reduce_vec > /dev/null
$P "$D/tree_pmc_FETCH_SIZE" "$D/tree_pmc_WRITE_SIZE" tree_f32_sum_8leaves_64MiB 603979776 - k_reduce_tree > /dev/null
$P "$D/vec1_pmc_FETCH_SIZE" "$D/vec1_pmc_WRITE_SIZE" reduce_f32_sum_m1_oop_128MiB 402653184 - "k_reduce_vec<0, 0, 1," > /dev/null
$P "$D/vec3_pmc_FETCH_SIZE" "$D/vec3_pmc_WRITE_SIZE" reduce_f32_sum_m3_oop_64MiB 335544320 - "k_reduce_vec<0, 0, 3," > /dev/null
for nl in 4 2; do
  if [ -d "$D/tree${nl}_pmc_FETCH_SIZE" ]; then
    # a streaming 2-leaf tree runs on the bucket kernel (reduce_tree.hip routes it, round 6)
    k=k_reduce_tree; [ $nl = 2 ] && k="k_reduce_vec<0, 0, 1,"
    $P "$D/tree${nl}_pmc_FETCH_SIZE" "$D/tree${nl}_pmc_WRITE_SIZE" "tree_f32_sum_${nl}leaves_64MiB" $(( (nl + 1) * 64 * 1048576 )) - "$k" > /dev/null
  fi
done
python3 -c "
import json; d = json.load(open('profiles/pmc_latest.json'))
for k, v in d['kernels'].items(): print(f\"{k:34s} {v['traffic_over_algorithmic']:.5f}  {v['kernel_symbol']}  {v['sources_sha256_16']}\")"
