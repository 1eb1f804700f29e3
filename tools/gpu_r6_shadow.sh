#!/bin/bash
# Weight-shadow pack: kernel tests, the large-H LSTM / GRU suites that read
# the shadows, the char-LM bench and its glue trace.
set -o pipefail
mkdir -p gpurun_out/shadow
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_shadow.py \
  tests/test_gpu_lstm_large.py tests/test_gpu_lstm_persist.py tests/test_gpu_gru_large.py tests/test_gpu_train.py tests/test_gpu_kernels.py \
  > gpurun_out/shadow/tests.log 2>&1 || { tail -40 gpurun_out/shadow/tests.log; exit 1; }
tail -2 gpurun_out/shadow/tests.log
timeout -k 10 240 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 > gpurun_out/shadow/charlm.log 2>&1 \
  || { tail -20 gpurun_out/shadow/charlm.log; exit 1; }
tail -1 gpurun_out/shadow/charlm.log | cut -c1-300
timeout -k 10 240 python tools/charlm_glue_trace.py > gpurun_out/shadow/charlm_glue.txt 2>&1 \
  || { tail -20 gpurun_out/shadow/charlm_glue.txt; exit 1; }
head -30 gpurun_out/shadow/charlm_glue.txt
