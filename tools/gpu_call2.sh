# leaf-2 tree A/B (ACC0 on / off, alternating) and the GPU-holding-parent A/B for the multi-rank launches
set -u -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/c2; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/leaf2_ab.py --rounds 2 > $O/leaf2_off_$r.jsonl 2> $O/leaf2_off_$r.err || exit $?
  CHR_TREE_ACC0=1 timeout -k 10 300 python -u tools/leaf2_ab.py --rounds 2 > $O/leaf2_acc0_$r.jsonl 2> $O/leaf2_acc0_$r.err || exit $?
done
for r in 1 2; do
  timeout -k 10 120 python -u tools/mpi_timing.py selftest intra_scatter_radix_batch 8 2 4 3 > $O/t_isc8_free_$r.txt 2>&1 || exit $?
  timeout -k 10 120 python -u tools/mpi_timing.py bin chiara_reduce_scatter 8 2 --overwrite b=4 base=1000 mem=device dtype=f32 reps=3 pattern=cancel > $O/t_rs8_free_$r.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/hold_queues.py 150 > $O/hold.txt 2>&1 &
HOLD=$!
for i in $(seq 60); do grep -q holding $O/hold.txt 2>/dev/null && break; sleep 1; done
for r in 1 2; do
  timeout -k 10 120 python -u tools/mpi_timing.py selftest intra_scatter_radix_batch 8 2 4 3 > $O/t_isc8_held_$r.txt 2>&1 || { kill $HOLD; exit 1; }
  timeout -k 10 120 python -u tools/mpi_timing.py bin chiara_reduce_scatter 8 2 --overwrite b=4 base=1000 mem=device dtype=f32 reps=3 pattern=cancel > $O/t_rs8_held_$r.txt 2>&1 || { kill $HOLD; exit 1; }
done
kill $HOLD; wait $HOLD
echo done
