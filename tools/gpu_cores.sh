#!/bin/bash
# Co-residency of RCCL's kernel with the streaming reductions (tools/coresidency_probe.cpp).
#   gpurun -- bash tools/gpu_cores.sh TAG "CONFIG1" "CONFIG2" ...
# A CONFIG is "name|env assignments|probe args"; each runs under rocprofv3 --kernel-trace, twice:
# the executable (ROCm 7.2 RCCL) and the Python host (torch's RCCL); tools/coresidency_report.py
# summarises each trace into gpurun_out/$TAG/report.jsonl.
set -u -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for cfg in "$@"; do
  IFS='|' read -r name envs args <<< "$cfg"
  for host in exe py; do
    if [ $host = exe ]; then cmd=(tools/coresidency_probe); else cmd=(python3 tools/coresidency_probe.py); fi
    d=$O/${name}_$host
    env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$d -o run -- "${cmd[@]}" $args \
      > $d.jsonl 2> $d.err
    rc=$?
    echo "$name $host rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $d.err; exit $rc; fi
    python3 tools/coresidency_report.py $d/run_kernel_trace.csv ${name}_$host >> $O/report.jsonl
    grep summary $O/report.jsonl | tail -1
  done
done
echo DONE
