#!/bin/bash
# oracle/selftests.sh -- TEST INFRASTRUCTURE ONLY, container-only (reads /root/reference).
#
# The reference keeps a DEBUG_MODE self-test main in most of its algorithm files.  Each
# file below is compiled unchanged with -DDEBUG_MODE (plus -include cmath -include algorithm: the DEBUG mains
# of reduce_scatter_{radix,pairwise}.cpp call std::max({...}) without <algorithm>, and
# all_reduce_radix_batch.cpp has `#include <cmath>` commented out, :8), twice:
#   _ref/selftest_<name>_mpi  as it is, against MPICH: the expected output (tests/golden/gen_selftests.py)
#   _ref/selftest_<name>      the same object with the file's algorithm function made a weak symbol
#                             (objcopy --weaken-symbol), linked with the reference-signature shim, whose
#                             strong definition on libchiara then serves the file's own main (travels to
#                             the GPU box; tests/test_gpu_ref_harness.py)
# -fno-inline keeps main's call a relocation against the symbol, which the link then binds to the shim.
# Not built: reduce_scatter_recursive_doubling.cpp's DEBUG main passes int* / double* where its own
# MPICH_reduce_scatter_rec_doubling takes const char* (:207, :222, :237, :252) and does not compile; its
# function is covered by the golden vectors and by testing/mpich_implementations/reduce_scatter/main.cpp.
set -euo pipefail
cd "$(dirname "$0")"
REF=${REF:-/root/reference}
MPICXX=${MPICXX:-/opt/conda/bin/mpicxx}
PKG=../configurable-hierarchical-allreduce-algorithms_amd
ROCM=${ROCM:-/opt/rocm}
MPI_HOME=${MPI_HOME:-/opt/conda}
SHIM=$PKG/csrc/shim/chiara_mpi_shim.cpp
LIB=$PKG/chiara_amd/libchiara.so
mkdir -p _ref

# name  source (under $REF)  function the shim replaces
while read -r name src fn; do
    [ -z "$name" ] && continue
    obj=_ref/selftest_$name.o
    if [ ! -f "$obj" ] || [ "$REF/$src" -nt "$obj" ] || [ "$0" -nt "$obj" ]; then
        MPICH_CXX=g++ $MPICXX -O1 -fno-inline -std=c++17 -include cmath -include algorithm -DDEBUG_MODE -w -c -o "$obj" "$REF/$src"
    fi
    if [ ! -f "_ref/selftest_${name}_mpi" ] || [ "$obj" -nt "_ref/selftest_${name}_mpi" ]; then
        MPICH_CXX=g++ $MPICXX -static-libstdc++ -o "_ref/selftest_${name}_mpi" "$obj"
    fi
    out=_ref/selftest_$name
    if [ ! -f "$out" ] || [ "$obj" -nt "$out" ] || [ "$SHIM" -nt "$out" ] || [ "$LIB" -nt "$out" ]; then
        sym=$(nm "$obj" | awk -v p="_Z${#fn}${fn}" '$2 == "T" && index($3, p) == 1 {print $3}')
        [ "$(echo "$sym" | wc -w)" = 1 ] || { echo "selftests: $fn: expected one definition, got '$sym'" >&2; exit 1; }
        objcopy --weaken-symbol="$sym" "$obj" "$out.weak.o"
        g++ -O2 -std=c++17 -I../include -I$ROCM/include -I$MPI_HOME/include -D__HIP_PLATFORM_AMD__ -o "$out" \
            "$out.weak.o" "$SHIM" -L$PKG/chiara_amd -lchiara -L$ROCM/lib -lamdhip64 $MPI_HOME/lib/libmpi.so \
            -Wl,-rpath,'$ORIGIN/../'$PKG/chiara_amd -Wl,-rpath,/usr/lib/x86_64-linux-gnu -Wl,-rpath,$ROCM/lib \
            -Wl,-rpath,$MPI_HOME/lib
        rm -f "$out.weak.o"
    fi
done <<'SPECS'
intra_reduce_scatter_radix testing/custom_implementations/work_dir/reduce_scatter/intra_reduce_scatter_radix.cpp intra_reduce_scatter_radix_batch
inter_linear_reduce testing/custom_implementations/work_dir/reduce_scatter/inter_linear_reduce.cpp inter_reduce_linear
intra_scatter_radix_batch testing/custom_implementations/work_dir/reduce_scatter/intra_scatter_radix_batch.cpp intra_scatter_radix_batch
all_reduce_radix_batch Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp all_reduce_radix_batch
reduce_scatter_radix testing/mpich_implementations/reduce_scatter/reduce_scatter_radix.cpp MPICH_reduce_scatter_radix
reduce_scatter_recursive_halving testing/mpich_implementations/reduce_scatter/reduce_scatter_recursive_halving.cpp MPICH_reduce_scatter_rec_halving
reduce_scatter_pairwise testing/mpich_implementations/reduce_scatter/reduce_scatter_pairwise.cpp MPICH_reduce_scatter_pairwise
allreduce_ring testing/mpich_implementations/all_reduce/allreduce_ring.cpp MPICH_Allreduce_ring
allreduce_recursive_doubling testing/mpich_implementations/all_reduce/allreduce_recursive_doubling.cpp MPICH_Allreduce_recursive_doubling
allreduce_reduce_scatter_allgather testing/mpich_implementations/all_reduce/allreduce_reduce_scatter_allgather.cpp MPICH_Allreduce_reduce_scatter_allgather
allreduce_recexch testing/mpich_implementations/all_reduce/allreduce_recexch.cpp MPICH_Allreduce_recursive_exchange
allreduce_k_reduce_scatter_allgather testing/mpich_implementations/all_reduce/allreduce_k_reduce_scatter_allgather.cpp MPICH_Allreduce_k_reduce_scatter_allgather
allreduce_recursive_multiplying testing/mpich_implementations/all_reduce/allreduce_recursive_multiplying.cpp MPICH_Allreduce_recursive_multiplying
SPECS
