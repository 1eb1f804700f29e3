# one-pass slab reduction (+ Adam): correctness + A/B against the two-pass tail
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py tests/test_gpu_multirank.py -x -v --timeout 120 --timeout-method thread > gpurun_out/op_tests.log 2>&1 || { tail -40 gpurun_out/op_tests.log; exit 1; }
tail -2 gpurun_out/op_tests.log
for b in 180 1440; do
  for v in 0 1; do
    PDRNN_ONE_PASS_REDUCE=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch $b > gpurun_out/op_b${b}_v$v.log 2>&1
    echo "B=$b one_pass=$v $(tail -1 gpurun_out/op_b${b}_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
for v in 0 1; do
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_ONE_PASS_REDUCE=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch 180 > gpurun_out/op_sync_v$v.log 2>&1
  echo "synced B=180 one_pass=$v $(tail -1 gpurun_out/op_sync_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  PDRNN_ONE_PASS_REDUCE=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --cell gru > gpurun_out/op_gru_v$v.log 2>&1
  echo "GRU B=1440 one_pass=$v $(tail -1 gpurun_out/op_gru_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/prof_op -o run -- python3 bench.py --steps 50 --warmup 10 --global-batch 180 > gpurun_out/op_prof.log 2>&1
db=$(find /tmp/prof_op -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/op_b180_kernel_stats.md
python tools/prof_seq.py "$db" lstm_small_step_gs_kernel 210 2 > gpurun_out/op_b180_seq.txt
cat gpurun_out/op_b180_seq.txt
