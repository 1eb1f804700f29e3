# large-H step loops as cached HIP graphs: tests, then char-LM / bi-LSTM / fp32 H=128 with and without
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py tests/test_gpu_coverage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lg_tests.log 2>&1 || { tail -40 gpurun_out/lg_tests.log; exit 1; }
tail -1 gpurun_out/lg_tests.log
for G in 0 1; do
  PDRNN_LARGE_GRAPH=$G timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 2 > gpurun_out/lg_charlm_g$G.log 2>&1
  tail -1 gpurun_out/lg_charlm_g$G.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('charlm graph=$G', d['value'], d['ms_per_step'])"
  PDRNN_LARGE_GRAPH=$G timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 > gpurun_out/lg_h128_g$G.log 2>&1
  tail -1 gpurun_out/lg_h128_g$G.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp32 h128 graph=$G', d['value'], d['ms_per_step'])"
done
PDRNN_LARGE_GRAPH=1 timeout -k 10 500 python bench/lm_bench.py --config bilstm --steps 3 --warmup 1 > gpurun_out/lg_bilstm_g1.log 2>&1
tail -1 gpurun_out/lg_bilstm_g1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bilstm graph=1', d['value'], d['ms_per_step'])"
