# Large-H LSTM/GRU numerics + secondary benchmarks (gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gru_large.py tests/test_gpu_lstm_large.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_large.log 2>&1 || exit 1
timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 3 --warmup 1 > gpurun_out/lm_bilstm.log 2>&1 || exit 2
timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 5 --warmup 2 > gpurun_out/lm_charlm.log 2>&1 || exit 3
