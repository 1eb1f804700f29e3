# one-launch fused step (fwd + head/CE + BPTT): correctness + A/B against two launches
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ol_tests.log 2>&1 || { tail -40 gpurun_out/ol_tests.log; exit 1; }
tail -2 gpurun_out/ol_tests.log
for b in 180 360 96; do
  for v in 0 1; do
    PDRNN_STEP_ONE_LAUNCH=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch $b > gpurun_out/ol_b${b}_v$v.log 2>&1
    echo "B=$b one_launch=$v $(tail -1 gpurun_out/ol_b${b}_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
for v in 0 1; do
  PDRNN_STEP_ONE_LAUNCH=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch 180 --cell gru > gpurun_out/ol_gru_v$v.log 2>&1
  echo "GRU B=180 one_launch=$v $(tail -1 gpurun_out/ol_gru_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_STEP_ONE_LAUNCH=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch 180 > gpurun_out/ol_sync_v$v.log 2>&1
  echo "synced B=180 one_launch=$v $(tail -1 gpurun_out/ol_sync_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/ol_b1440.log 2>&1
echo "B=1440 $(tail -1 gpurun_out/ol_b1440.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
