set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xo_tests.log 2>&1 || { tail -40 gpurun_out/xo_tests.log; exit 1; }
tail -1 gpurun_out/xo_tests.log
for i in 1 2; do
for b in 180 360; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch $b > gpurun_out/xo_b${b}.log 2>&1
  echo "B=$b $(tail -1 gpurun_out/xo_b${b}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch 180 --cell gru > gpurun_out/xo_gru.log 2>&1
echo "GRU B=180 $(tail -1 gpurun_out/xo_gru.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
