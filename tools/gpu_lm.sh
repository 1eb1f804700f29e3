# large-H path (one gpurun call): GEMM / large-LSTM / GRU / persistent-recurrence
# tests, char-LM with each persistent-verification mode, bi-LSTM
#   tools/gpu_lm.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-lm}
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py tests/test_gpu_lstm_persist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for v in 0 1 2; do
  PDRNN_LSTM_PERSIST_VERIFY=$v timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 > gpurun_out/${tag}_charlm_verify$v.log 2>&1 || { tail -20 gpurun_out/${tag}_charlm_verify$v.log; exit 1; }
  echo "verify=$v $(tail -1 gpurun_out/${tag}_charlm_verify$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['persist_verify'], d['persist_fallbacks'])")"
done
timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 6 --warmup 2 > gpurun_out/${tag}_bilstm.log 2>&1 || { tail -20 gpurun_out/${tag}_bilstm.log; exit 1; }
echo "bilstm $(tail -1 gpurun_out/${tag}_bilstm.log | cut -c1-200)"
