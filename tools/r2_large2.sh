set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r2l2_tests.log 2>&1 || { tail -40 gpurun_out/r2l2_tests.log; exit 1; }
tail -1 gpurun_out/r2l2_tests.log
timeout -k 10 600 python bench/lm_bench.py --config bilstm --batch 4096 --steps 5 --warmup 2 > gpurun_out/r2l2_bilstm_b4096.log 2>&1
tail -1 gpurun_out/r2l2_bilstm_b4096.log | cut -c1-250
timeout -k 10 600 python bench/lm_bench.py --config charlm --batch 128 --steps 10 --warmup 2 > gpurun_out/r2l2_charlm_b128.log 2>&1
tail -1 gpurun_out/r2l2_charlm_b128.log | cut -c1-250
