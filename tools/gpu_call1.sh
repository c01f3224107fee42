set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/c1; mkdir -p $O
timeout -k 10 60 tools/nan_invalid_probe > $O/nan_invalid.txt 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_nan_payloads.py tests/test_gpu_kernels.py -k "nan or complex or pair" > $O/pytest_nan.txt 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do timeout -k 10 120 python -u tools/mpi_timing.py selftest intra_scatter_radix_batch 8 2 4 3 > $O/t_isc8_$i.txt 2>&1 || exit $?; done
timeout -k 10 120 python -u tools/mpi_timing.py selftest intra_reduce_scatter_radix 9 2 2 3 > $O/t_irs9.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/mpi_timing.py bin chiara_reduce_scatter 8 2 --overwrite b=4 base=1000 mem=device dtype=f32 reps=3 pattern=cancel > $O/t_rs8.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/mpi_timing.py bin chiara_allreduce 8 2 --overwrite b=4 base=4096 mem=device dtype=f32 reps=3 pattern=cancel > $O/t_ar8.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/leaf2_ab.py --rounds 2 > $O/leaf2_ab.jsonl 2> $O/leaf2_ab.err || exit $?
echo done
