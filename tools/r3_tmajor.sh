set -e
export TMPDIR=/tmp
PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch 1440 > gpurun_out/r3k_base.log 2>&1
PDRNN_DIAG_TMAJOR=1 PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch 1440 > gpurun_out/r3k_tmajor.log 2>&1 || true
grep -A1 "fwd(head step) grid=1440" gpurun_out/r3k_base.log | tail -2
grep -A1 "fwd(head step) grid=1440" gpurun_out/r3k_tmajor.log | tail -2
