#!/bin/bash
# Round 2, GPU call F: PMC passes on the m=3 bucket reduction at 512 MiB vs 1 GiB (VERDICT r1
# item 3), one rocprofv3 run per counter group (TCP address translation, TA stalls, TCC/EA).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P="python3 tools/mstream_probe.py --ms 3,7 --mib 256,512,1024 --layouts sep --reps 6"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_ms -o trace -- $P \
  > gpurun_out/pmc_ms_trace.jsonl 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
  TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_ms -o utcl1 -- $P > gpurun_out/pmc_ms_utcl1.jsonl 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum \
  TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum \
  TCP_UTCL1_THRASHING_STALL_sum GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_ms -o stall -- $P > gpurun_out/pmc_ms_stall.jsonl 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum \
  TCC_EA0_WRREQ_STALL_sum TCC_LATENCY_FIFO_FULL_sum GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_ms -o tcc -- $P > gpurun_out/pmc_ms_tcc.jsonl 2>&1
