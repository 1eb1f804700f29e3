# persistent large-H recurrence: numerics vs per-step + torch, then char-LM B=128 with / without
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_persist.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_persist_tests.log 2>&1
tail -3 gpurun_out/r2_persist_tests.log
timeout -k 10 200 python -u bench/lm_bench.py --config charlm --steps 5 --warmup 2 > gpurun_out/r2_persist_charlm.log 2>&1
tail -1 gpurun_out/r2_persist_charlm.log
PDRNN_LSTM_PERSIST=0 timeout -k 10 200 python -u bench/lm_bench.py --config charlm --steps 5 --warmup 2 > gpurun_out/r2_persist_charlm_off.log 2>&1
tail -1 gpurun_out/r2_persist_charlm_off.log
