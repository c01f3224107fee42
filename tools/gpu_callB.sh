# Final PMC and kernel-duration records for the tree and out-of-place fold entries, one GPU's own C4 / C5 grids at
# the in-collective cap, and the 2-leaf tree vs the bucket kernel under rocprof
set -u -o pipefail
bash tools/gpu.sh treepmc vecpmc ranktrees12 || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/leaf2_prof" -o run \
  -- python3 tools/leaf2_ab.py --rounds 1 > gpurun_out/leaf2_prof.jsonl 2> gpurun_out/leaf2_prof.err || exit $?
echo done
