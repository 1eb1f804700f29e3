# BPTT lanes per unit (L = 4 vs 8) at the per-GPU batches of N = 8/4/2/1
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 180 360 720 1440; do
  for L in 4 8; do
    PDRNN_LSTM_BWD_L=$L timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/ls_b${B}_L$L.log 2>&1
    tail -1 gpurun_out/ls_b${B}_L$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B L=$L', d['value'], d['ms_per_step'])"
  done
done
PDRNN_LSTM_BWD_L=8 timeout -k 10 120 python bench/stamps.py 180 > gpurun_out/ls_stamps_L8.log 2>&1
grep -E "stamps" gpurun_out/ls_stamps_L8.log | sort -u | head -4
