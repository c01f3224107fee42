# A/B of the user-op fold kernel's compile-time knobs (include/chiara_user_op.hpp): every
# tests/userop/libhalfadd_u*.so variant through tools/userop_bench.py, 2 alternating rounds -> gpurun_out/userop_ab.jsonl.
# Variants are built beforehand, on the CPU, e.g. for U in 1 2 4 8:
#   hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -ffp-contract=off -DCHR_USER_FOLD_U=$U -Iinclude \
#     -o tests/userop/libhalfadd_u$U.so tests/userop/halfadd_op.hip
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for so in tests/userop/libhalfadd_u*.so; do
    CHR_USEROP_SO=$PWD/$so timeout -k 10 120 python tools/userop_bench.py >> gpurun_out/userop_ab.jsonl || exit $?
  done
done
echo done
