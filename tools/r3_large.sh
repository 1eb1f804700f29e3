# large-H path on the in-tree GEMM: numerics tests, then char-LM / bi-LSTM A/B vs the library GEMMs
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for cfg in charlm bilstm; do
  for g in mfma torch; do
    PDRNN_GEMM=$g timeout -k 10 300 python bench/lm_bench.py --config $cfg --steps 4 --warmup 1 > gpurun_out/${tag}_${cfg}_$g.log 2>&1 || { tail -20 gpurun_out/${tag}_${cfg}_$g.log; exit 1; }
    echo "$cfg $g $(tail -1 gpurun_out/${tag}_${cfg}_$g.log | cut -c1-160)"
  done
done
