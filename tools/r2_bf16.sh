set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || { tail -40 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
timeout -k 10 120 python bench.py --layers 1 --dtype bf16 --steps 200 --warmup 20 > gpurun_out/bf16k_1x32.log 2>&1
echo "1x32 bf16 $(tail -1 gpurun_out/bf16k_1x32.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
timeout -k 10 120 python bench.py --dtype bf16 --steps 200 --warmup 20 > gpurun_out/bf16k_2x32.log 2>&1
echo "2x32 bf16 $(tail -1 gpurun_out/bf16k_2x32.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
timeout -k 10 120 python bench.py --dtype bf16 --steps 200 --warmup 20 --global-batch 180 > gpurun_out/bf16k_b180.log 2>&1
echo "2x32 bf16 B=180 $(tail -1 gpurun_out/bf16k_b180.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
