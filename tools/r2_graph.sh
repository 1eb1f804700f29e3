# graph-replayed synced step: comm tests, then eager vs graph at the 8-GPU per-rank batch
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -60 gpurun_out/graph_tests.log; exit 1; }
tail -1 gpurun_out/graph_tests.log
for B in 180 720; do
  for G in 0 1; do
    PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 PDRNN_CUDA_GRAPH=$G timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/graph_b${B}_g$G.log 2>&1
    tail -1 gpurun_out/graph_b${B}_g$G.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B graph=$G', d['value'], d['ms_per_step'])"
  done
done
