# large-H path: numerics tests, then char-LM / bi-LSTM benches
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3lm}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for cfg in charlm bilstm; do
  timeout -k 10 300 python bench/lm_bench.py --config $cfg --steps 6 --warmup 2 > gpurun_out/${tag}_${cfg}.log 2>&1 || { tail -20 gpurun_out/${tag}_${cfg}.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/${tag}_${cfg}.log | cut -c1-200)"
done
