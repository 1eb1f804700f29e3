set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_train.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ring_tests.log 2>&1 || { tail -40 gpurun_out/ring_tests.log; exit 1; }
tail -1 gpurun_out/ring_tests.log
for i in 1 2; do
  PDRNN_CUDA_GRAPH=1 PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --global-batch 180 --steps 300 --warmup 30 > gpurun_out/ring_g180.log 2>&1
  echo "graph synced B=180 $(tail -1 gpurun_out/ring_g180.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
done
PDRNN_CUDA_GRAPH=1 PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --global-batch 720 --steps 300 --warmup 30 > gpurun_out/ring_g720.log 2>&1
echo "graph synced B=720 $(tail -1 gpurun_out/ring_g720.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
PDRNN_CUDA_GRAPH=1 PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --global-batch 360 --steps 300 --warmup 30 > gpurun_out/ring_g360.log 2>&1
echo "graph synced B=360 $(tail -1 gpurun_out/ring_g360.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
