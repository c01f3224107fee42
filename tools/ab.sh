#!/bin/bash
# Product-API A/B runs behind the occupancy-cap and XCD-run policy, on the GPU box:
#   gpurun -- bash tools/ab.sh cap    C2 / mstream m=3,7 / collective-kernel rows vs CHR_WG_PER_CU_{VEC,TREE}
#   gpurun -- bash tools/ab.sh runs   C2 with the policy XCD map vs 256 KiB runs, 3 alternating rounds
#   gpurun -- bash tools/ab.sh hand   C2 / mstream with the odd-XCD handover off / at shifts 5-6
#   gpurun -- bash tools/ab.sh handtree   the in-collective tree rows with the handover off / on
# Results land under gpurun_out/cap/ or gpurun_out/ab_runs/ (copied to profiles/r02/occupancy_cap/, ab_runs/).
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
frac() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'], d['roofline']['frac'])" "$1"; }
case "${1:-}" in
cap)
  mkdir -p gpurun_out/cap
  for r in 1 2; do
    for c in 0 10 12 14 16; do
      CHR_WG_PER_CU_VEC=$c timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
        > gpurun_out/cap/c2_cap${c}_r${r}.json 2>/dev/null || exit 1
      echo "c2 cap=$c r=$r $(frac gpurun_out/cap/c2_cap${c}_r${r}.json)"
    done
  done
  for c in 0 12 10; do
    CHR_WG_PER_CU_VEC=$c timeout -k 10 300 python tools/mstream_probe.py --ms 3,7 --mib 256 --layouts sep --sets 1,8 \
      > gpurun_out/cap/mstream_cap${c}.jsonl 2>/dev/null || exit 1
    echo "mstream cap=$c"; cut -c1-300 gpurun_out/cap/mstream_cap${c}.jsonl
  done
  for c in 0 8 10 12; do
    CHR_WG_PER_CU_TREE=$c timeout -k 10 400 python bench.py --collective-kernels > gpurun_out/cap/ck_tree_cap${c}.json \
      2>/dev/null || exit 1
    echo "tree cap=$c $(python -c "import json;d=json.load(open('gpurun_out/cap/ck_tree_cap${c}.json'))['collective_kernels']['rows'];print({k: v['frac'] for k, v in d.items()})")"
  done ;;
runs)
  mkdir -p gpurun_out/ab_runs
  for r in 1 2 3; do
    for v in policy 256; do
      if [ "$v" = policy ]; then unset CHR_XCD_RUN_KIB; else export CHR_XCD_RUN_KIB=$v; fi
      timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
        > gpurun_out/ab_runs/c2_${v}_r${r}.json 2>/dev/null || exit 1
      echo "c2 runs=$v r=$r $(frac gpurun_out/ab_runs/c2_${v}_r${r}.json)"
    done
  done ;;
hand)  # the odd-XCD handover (xcd_trip_w): off (shift 0) / policy (6) / 5 / 7, C2 at 20 and 200 steps, mstream m=3,7
  mkdir -p gpurun_out/ab_hand
  for r in 1 2 3; do
    for v in 0 6 5; do
      CHR_XCD_HAND_SHIFT=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
        > gpurun_out/ab_hand/c2_shift${v}_r${r}.json 2>/dev/null || exit 1
      CHR_XCD_HAND_SHIFT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/ab_hand/c2s20_shift${v}_r${r}.json 2>/dev/null || exit 1
      echo "c2 shift=$v r=$r $(frac gpurun_out/ab_hand/c2_shift${v}_r${r}.json)   s20 $(frac gpurun_out/ab_hand/c2s20_shift${v}_r${r}.json)"
    done
  done
  for v in 0 6; do
    CHR_XCD_HAND_SHIFT=$v timeout -k 10 300 python tools/mstream_probe.py --ms 3,7 --mib 256 --layouts sep --sets 1,8 \
      > gpurun_out/ab_hand/mstream_shift${v}.jsonl 2>/dev/null || exit 1
    echo "mstream shift=$v"; cut -c1-300 gpurun_out/ab_hand/mstream_shift${v}.jsonl
  done ;;
gate)  # bench.py's untimed gate kernel ahead of the C2 timed region: off / on at the driver's 20 / 5 and at 200 / 20
  mkdir -p gpurun_out/ab_gate
  for r in 1 2 3 4; do
    for v in 0 1; do
      CHR_BENCH_GATE=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/ab_gate/c2s20_gate${v}_r${r}.json 2>/dev/null || exit 1
      CHR_BENCH_GATE=$v timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
        > gpurun_out/ab_gate/c2s200_gate${v}_r${r}.json 2>/dev/null || exit 1
      echo "c2 gate=$v r=$r s20 $(frac gpurun_out/ab_gate/c2s20_gate${v}_r${r}.json)  s200 $(frac gpurun_out/ab_gate/c2s200_gate${v}_r${r}.json)"
    done
  done ;;
handtree)  # the odd-XCD handover on the tree kernel: in-collective rows (rank-alone replays = one GPU's grids)
  mkdir -p gpurun_out/ab_hand
  for r in 1 2; do
    for v in ${SHIFTS:-0 6}; do  # "def": the library default (no env)
      if [ "$v" = def ]; then unset CHR_XCD_HAND_SHIFT; else export CHR_XCD_HAND_SHIFT=$v; fi
      timeout -k 10 400 python bench.py --collective-kernels \
        > gpurun_out/ab_hand/ck_shift${v}_r${r}.json 2>/dev/null || exit 1
      echo "tree shift=$v r=$r $(python -c "import json;d=json.load(open('gpurun_out/ab_hand/ck_shift${v}_r${r}.json'))['collective_kernels']['rows'];print({k: v['frac'] for k, v in d.items()})")"
    done
  done ;;
handtreebench)  # the tree handover on tools/tree_bench.py (one tree at 8 / 64 / 128 MiB pieces, batched C4 slices)
  mkdir -p gpurun_out/ab_hand
  for r in 1 2; do
    for v in ${SHIFTS:-def 6 0}; do
      if [ "$v" = def ]; then unset CHR_XCD_HAND_SHIFT; else export CHR_XCD_HAND_SHIFT=$v; fi
      timeout -k 10 300 python tools/tree_bench.py > gpurun_out/ab_hand/tb_shift${v}_r${r}.json 2>/dev/null || exit 1
      echo "tree_bench shift=$v r=$r $(python -c "
import json; d = json.load(open('gpurun_out/ab_hand/tb_shift${v}_r${r}.json'))
a = {k: round(v['tree']['alg_GBps'] / 8000, 4) for k, v in d['tree_vs_folds_c4']['f32'].items()}
b = {k: (v['batched_cold']['frac'], v['batched_warm']['frac']) for k, v in d['slice_batched_c4']['f32'].items()}
print(a, b)")"
    done
  done ;;
tree)  # the tree shape: policy vs the previous one (16 per CU, 512 KiB runs), collective-kernel rows, alternating
  mkdir -p gpurun_out/ab_tree
  for r in 1 2; do
    for v in prev policy; do
      if [ "$v" = prev ]; then export CHR_WG_PER_CU_TREE=16 CHR_XCD_RUN_KIB=512; else unset CHR_WG_PER_CU_TREE CHR_XCD_RUN_KIB; fi
      timeout -k 10 400 python bench.py --collective-kernels > gpurun_out/ab_tree/ck_${v}_r${r}.json 2>/dev/null || exit 1
      echo "tree $v r=$r $(python -c "import json;d=json.load(open('gpurun_out/ab_tree/ck_${v}_r${r}.json'))['collective_kernels']['rows'];print({k[:-0 or None]: v['frac'] for k, v in d.items() if 'copies' not in k})")"
    done
  done
  unset CHR_WG_PER_CU_TREE CHR_XCD_RUN_KIB ;;
mid)  # mid-size buckets: streaming shape (nt, one wave) vs plain 256-thread at 4-64 MiB,
      # m = 1 and 3, the sweep's rotation (16 sets) and an HBM-cold one (>= 2 GiB), gated, 3 alternating rounds
  mkdir -p gpurun_out/ab_mid
  for r in 1 2 3; do
    for v in 0 1; do
      for rot in "--sets 16" "--ws-mib 2048"; do
        tag="nt${v}_$(echo $rot | tr -d ' -')_r${r}"
        CHR_REDUCE_NT=$v timeout -k 10 200 python tools/mstream_probe.py --ms 1,3 --mib 4,8,16,32,64 --layouts sep \
          $rot --reps 200 --gate --tag "$tag" >> gpurun_out/ab_mid/mid.jsonl 2>>gpurun_out/ab_mid/mid.err || exit 1
        echo "mid $tag done"
      done
    done
  done ;;
mid2)  # follow-ups of `mid`: the cache-resident case (1-2 sets), the streaming shape's cap / XCD runs / hand at
       # 8-32 MiB, and the HIP runtime's kernel fence options (what the inter-launch gap is made of)
  mkdir -p gpurun_out/ab_mid
  P="python tools/mstream_probe.py --layouts sep --reps 200 --gate"
  for r in 1 2; do
    for v in 0 1; do
      CHR_REDUCE_NT=$v timeout -k 10 200 $P --ms 1,3 --mib 4,8,16,32,64 --sets 1,2 --tag "warm_nt${v}_r${r}" \
        >> gpurun_out/ab_mid/mid2.jsonl 2>>gpurun_out/ab_mid/mid2.err || exit 1
    done
    for c in 0 12 16 24; do
      CHR_REDUCE_NT=1 CHR_WG_PER_CU_VEC=$c timeout -k 10 200 $P --ms 1,3 --mib 8,16,32 --ws-mib 2048 --tag "cap${c}_r${r}" \
        >> gpurun_out/ab_mid/mid2.jsonl 2>>gpurun_out/ab_mid/mid2.err || exit 1
    done
    for x in 0 256 1024; do
      CHR_REDUCE_NT=1 CHR_XCD_RUN_KIB=$x timeout -k 10 200 $P --ms 1,3 --mib 8,16,32 --ws-mib 2048 --tag "xrun${x}_r${r}" \
        >> gpurun_out/ab_mid/mid2.jsonl 2>>gpurun_out/ab_mid/mid2.err || exit 1
    done
    for h in 0 4; do
      CHR_REDUCE_NT=1 CHR_XCD_HAND_SHIFT=$h timeout -k 10 200 $P --ms 1,3 --mib 8,16,32 --ws-mib 2048 --tag "hand${h}_r${r}" \
        >> gpurun_out/ab_mid/mid2.jsonl 2>>gpurun_out/ab_mid/mid2.err || exit 1
    done
    for f in "AMD_OPT_FLUSH=0" "AMD_OPT_FLUSH=1" "DEBUG_CLR_SKIP_RELEASE_SCOPE=1"; do
      env CHR_REDUCE_NT=1 $f timeout -k 10 200 $P --ms 1 --mib 1,4,16,64 --ws-mib 2048 --tag "${f}_r${r}" \
        >> gpurun_out/ab_mid/mid2.jsonl 2>>gpurun_out/ab_mid/mid2.err || exit 1
    done
    echo "mid2 r=$r done"
  done ;;
xrun)  # the translation cliff: XCD run length vs working sets past the translation
       # caches' reach -- m = 1/3/7 at 1 GiB buckets (one set: every call walks 3-9 GiB) and 256 MiB rotated
       # over ~5 GiB; 512 KiB (policy for m >= 3), 2/4/8 MiB runs (each 2 MiB fragment on one XCD), identity
  mkdir -p gpurun_out/ab_xrun
  P="python tools/mstream_probe.py --layouts sep --reps 12 --gate"
  for r in 1 2; do
    for x in ${XRUNS:-512 2048 4096 8192 0}; do
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 $P --ms 1,3,7 --mib 1024 --sets 1 --tag "xrun${x}_1g_r${r}" \
        >> gpurun_out/ab_xrun/xrun.jsonl 2>>gpurun_out/ab_xrun/xrun.err || exit 1
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 $P --ms 3,7 --mib 256 --ws-mib 5120 --tag "xrun${x}_256m_ws5g_r${r}" \
        >> gpurun_out/ab_xrun/xrun.jsonl 2>>gpurun_out/ab_xrun/xrun.err || exit 1
      echo "xrun $x r=$r done"
    done
  done ;;
xrunpmc)  # translation counters beside the rates above: m = 3, 1 GiB, one set, policy vs 2 MiB runs
  mkdir -p gpurun_out/ab_xrun
  for x in 512 ${XRUN_PMC:-2048}; do
    CHR_XCD_RUN_KIB=$x timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
      GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d "$PWD/gpurun_out/ab_xrun/pmc_x$x" -o run \
      -- python3 tools/mstream_probe.py --layouts sep --reps 6 --ms 3 --mib 1024 --sets 1 \
      > gpurun_out/ab_xrun/pmc_x$x.txt 2>&1 || exit 1
    echo "xrunpmc $x done"
  done ;;
tlbpf)  # translation prefetch (CHR_TLB_PF_TRIPS: workgroups ahead; CHR_TLB_PF_PAGE_KIB: granule) past the
        # translation caches' reach, and C2 with it off (the policy) to check the code costs nothing there
  mkdir -p gpurun_out/ab_tlbpf
  P="python tools/mstream_probe.py --layouts sep --reps 12 --gate"
  for r in 1 2; do
    for v in ${PFS:-0 2816 5632 11264 2816/512 2816/64}; do
      pf=${v%%/*}; pg=2048; [ "$v" != "$pf" ] && pg=${v##*/}
      CHR_TLB_PF_TRIPS=$pf CHR_TLB_PF_PAGE_KIB=$pg timeout -k 10 300 $P --ms 1,3,7 --mib 1024 --sets 1 \
        --tag "pf${pf}_pg${pg}_1g_r${r}" >> gpurun_out/ab_tlbpf/pf.jsonl 2>>gpurun_out/ab_tlbpf/pf.err || exit 1
      CHR_TLB_PF_TRIPS=$pf CHR_TLB_PF_PAGE_KIB=$pg timeout -k 10 300 $P --ms 3 --mib 256 --ws-mib 5120 \
        --tag "pf${pf}_pg${pg}_256m_ws5g_r${r}" >> gpurun_out/ab_tlbpf/pf.jsonl 2>>gpurun_out/ab_tlbpf/pf.err || exit 1
      echo "tlbpf $v r=$r done"
    done
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_tlbpf/c2_r${r}.json \
      2>/dev/null || exit 1
    echo "c2 r=$r $(frac gpurun_out/ab_tlbpf/c2_r${r}.json)"
  done ;;
treebl)  # two-wave tree workgroups (CHR_TREE_BL=128, same waves per CU) and the
         # tree handover off, on the in-collective rows (rank-alone rows: one GPU's own grids, whole-call spans)
  mkdir -p gpurun_out/ab_treebl
  for r in 1 2; do
    for v in ${ARMS:-64_def 128_def 64_0 128_0}; do
      bl=${v%%_*}; h=${v##*_}
      if [ "$h" = def ]; then unset CHR_XCD_HAND_SHIFT; else export CHR_XCD_HAND_SHIFT=$h; fi
      CHR_TREE_BL=$bl timeout -k 10 400 python bench.py --collective-kernels > gpurun_out/ab_treebl/ck_${v}_r${r}.json \
        2>/dev/null || exit 1
      echo "treebl $v r=$r $(python -c "import json;d=json.load(open('gpurun_out/ab_treebl/ck_${v}_r${r}.json'))['collective_kernels']['rows'];print({k: (v['frac'], v.get('graph_replay', {}).get('eager', {}).get('frac')) for k, v in d.items() if 'rank0' in k})")"
    done
  done
  unset CHR_XCD_HAND_SHIFT ;;
xrun3)  # XCD runs for m = 2, 3 at mid sizes: 256 KiB vs the 512 KiB policy (m = 3) / identity (m = 2), 2 GiB rotation
  mkdir -p gpurun_out/ab_xrun
  P="python tools/mstream_probe.py --layouts sep --reps 100 --gate"
  for r in 1 2 3; do
    for x in 256 512 0; do
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 $P --ms 2,3 --mib 16,32,64,128,256 --ws-mib 2048 --tag "x${x}_r${r}" \
        >> gpurun_out/ab_xrun/xrun3.jsonl 2>>gpurun_out/ab_xrun/xrun3.err || exit 1
    done
    echo "xrun3 r=$r done"
  done ;;
wspmc)  # the working-set cliff's counters: m = 3 at 256 MiB over 1 set (1.25 GiB) vs 4 sets (5 GiB), two passes
  mkdir -p gpurun_out/ab_wspmc
  for sets in 1 4; do
    for pass in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
                "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum"; do
      tag=$(echo $pass | cut -d' ' -f1 | cut -d_ -f1)
      timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$PWD/gpurun_out/ab_wspmc/s${sets}_$tag" -o run \
        -- python3 tools/mstream_probe.py --layouts sep --reps 8 --ms 3 --mib 256 --sets $sets \
        > gpurun_out/ab_wspmc/s${sets}_$tag.txt 2>&1 || exit 1
      echo "wspmc sets=$sets $tag done"
    done
  done ;;
treerun)  # XCD runs of the 8-leaf trees (policy 512 KiB) on one GPU's own C4 / C5 grids, by rocprof kernel
          # duration (tools/rank_trees_summary.py), 2 alternating rounds
  mkdir -p gpurun_out/ab_treerun
  for r in 1 2; do
    for x in ${XRUNS:-512 256 1024}; do
      d="$PWD/gpurun_out/ab_treerun/x${x}_r${r}"
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
        -- python3 bench.py --rank-trees > "$d.json" 2>/dev/null || exit 1
      echo "treerun $x r=$r $(python tools/rank_trees_summary.py "$d.json" "$d" | python -c "
import json, sys; d = json.load(sys.stdin)['rank_trees_rocprof']; print({k.replace('_rank0_alone', ''): v['frac_avg'] for k, v in d.items()})")"
    done
  done ;;
treeu)  # U = 1 vs 2 for the floating 8-leaf trees (CHR_TREE_U: the knob exists at commit bace861 only) on one GPU's
        # own C4 / C5 grids, at the in-collective
        # cap 12 (CHR_WG_PER_CU_TREE=12, what CoresidentScope gives them beside RCCL) and at the standalone policy 16,
        # by rocprof kernel duration (tools/rank_trees_summary.py), 3 alternating rounds
  mkdir -p gpurun_out/ab_treeu
  for r in 1 2 3; do
    for c in 12 16; do
      for u in 1 2; do
        d="$PWD/gpurun_out/ab_treeu/c${c}_u${u}_r${r}"
        CHR_WG_PER_CU_TREE=$c CHR_TREE_U=$u timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
          -- python3 bench.py --rank-trees > "$d.json" 2>/dev/null || exit 1
        echo "treeu cap=$c u=$u r=$r $(python tools/rank_trees_summary.py "$d.json" "$d" | python -c "
import json, sys; d = json.load(sys.stdin)['rank_trees_rocprof']; print({k.replace('_rank0_alone', ''): v['frac_avg'] for k, v in d.items()})")"
      done
    done
  done ;;
treestage)  # the LDS-staged 8-leaf trees (CHR_TREE_STAGE: a round-5 working-tree knob, never committed; the
            # kernel is tools/reduce_microbench.hip's k_tree_lds) against the one-vector trip on one GPU's own C4 / C5 grids at
            # the in-collective cap 12, by rocprof kernel duration (tools/rank_trees_summary.py), 3 alternating rounds
  mkdir -p gpurun_out/ab_treestage
  for r in 1 2 3; do
    for v in 0 1; do
      d="$PWD/gpurun_out/ab_treestage/s${v}_r${r}"
      CHR_WG_PER_CU_TREE=12 CHR_TREE_STAGE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" \
        -o run -- python3 bench.py --rank-trees > "$d.json" 2>/dev/null || exit 1
      echo "treestage stage=$v r=$r $(python tools/rank_trees_summary.py "$d.json" "$d" | python -c "
import json, sys; d = json.load(sys.stdin)['rank_trees_rocprof']; print({k.replace('_rank0_alone', ''): v['frac_avg'] for k, v in d.items()})")"
    done
  done ;;
xrun4)  # XCD runs for wide fan-in (m = 4..7) and m = 3 at 1 GiB: 128 / 256 KiB vs the 512 KiB policy, 2 GiB rotation
  mkdir -p gpurun_out/ab_xrun
  P="python tools/mstream_probe.py --layouts sep --reps 40 --gate"
  for r in 1 2; do
    for x in 256 512 128; do
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 $P --ms 4,5,7 --mib 32,128,256 --ws-mib 2048 --tag "x${x}_r${r}" \
        >> gpurun_out/ab_xrun/xrun4.jsonl 2>>gpurun_out/ab_xrun/xrun4.err || exit 1
      CHR_XCD_RUN_KIB=$x timeout -k 10 300 $P --ms 3 --mib 1024 --sets 1 --reps 12 --tag "x${x}_1g_r${r}" \
        >> gpurun_out/ab_xrun/xrun4.jsonl 2>>gpurun_out/ab_xrun/xrun4.err || exit 1
    done
    echo "xrun4 r=$r done"
  done ;;
*) echo "usage: tools/ab.sh cap|runs|tree|mid|mid2|xrun|xrunpmc|tlbpf|treebl|xrun3|wspmc|treerun|xrun4|treeu|treestage"; exit 2 ;;
esac
echo AB_DONE
