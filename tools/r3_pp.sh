# ping-pong step kernels: numerics (forced at small shapes), then bi-LSTM A/B (pp vs GemmPipe tiles)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3pp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for pp in 1 0; do
  PDRNN_LSTM_LARGE_PP_BWD=$pp timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 4 --warmup 1 > gpurun_out/${tag}_bilstm_pp$pp.log 2>&1 || { tail -20 gpurun_out/${tag}_bilstm_pp$pp.log; exit 1; }
  echo "pp=$pp $(tail -1 gpurun_out/${tag}_bilstm_pp$pp.log | cut -c1-200)"
done
