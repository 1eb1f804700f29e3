# throughput backward (lstm_small_tp.hip): correctness tests, then an nb sweep
# over per-GPU batch sizes (N = 8/4/2/1 of the headline global batch 1440)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tp_tests.log 2>&1 || { tail -60 gpurun_out/tp_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/tp_tests.log | tail -3
for B in 1440 720 360 180; do
  for nb in 1 2 3; do
    PDRNN_LSTM_NB_BWD=$nb timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/tp_b${B}_nb${nb}.log 2>&1
    tail -1 gpurun_out/tp_b${B}_nb${nb}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B nb=$nb', d['value'], d['ms_per_step'])"
  done
done
for nb in 1 3; do
  PDRNN_LSTM_NB_BWD=$nb timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cell gru > gpurun_out/tp_gru_nb${nb}.log 2>&1
  tail -1 gpurun_out/tp_gru_nb${nb}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('GRU nb=$nb', d['value'], d['ms_per_step'])"
done
