# The 2-leaf tree and the out-of-place m = 1 fold at 64 MiB pieces under rocprofv3 kernel stats, at C2's rotation
# (1.9 GiB, DESIGN §4.1's warm side of the translation cliff) and at the PMC runs' 4.5 GiB -> gpurun_out/leaf2_rot*/
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rot in 1.9 4.5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/leaf2_rot$rot/tree2" -o run \
    -- python3 tools/tree_pmc.py 60 --leaves 2 --rot-gib $rot > gpurun_out/leaf2_rot$rot.tree2.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/leaf2_rot$rot/vec1" -o run \
    -- python3 tools/tree_pmc.py 60 --vec 1 --mib 64 --rot-gib $rot > gpurun_out/leaf2_rot$rot.vec1.log 2>&1 || exit $?
  echo "rot $rot done"
done
