# GPU tests, HIP-graph replay of the synced motion step vs eager at the 8-GPU per-rank
# batch (PDRNN_FORCE_GRAD_SYNC=1: RCCL all-reduce + Adam on one GPU), and the char-LM
# with the 8-unit split-K cell kernel vs the per-element one.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
: > gpurun_out/graph.log
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench/host_overhead.py --global-batch 180 >> gpurun_out/graph.log 2>&1 || exit 2
PDRNN_CUDA_GRAPH=1 PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench/host_overhead.py --global-batch 180 >> gpurun_out/graph.log 2>&1 || exit 3
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 180 >> gpurun_out/graph.log 2>&1 || exit 4
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 180 --cuda-graph >> gpurun_out/graph.log 2>&1 || exit 5
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 720 --cuda-graph >> gpurun_out/graph.log 2>&1 || exit 6
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 720 >> gpurun_out/graph.log 2>&1 || exit 7
: > gpurun_out/lm.log
PDRNN_LSTM_LARGE_CELL1=1 timeout -k 10 200 python bench/lm_bench.py --config charlm --steps 5 --warmup 2 >> gpurun_out/lm.log 2>&1 || exit 8
timeout -k 10 200 python bench/lm_bench.py --config charlm --steps 5 --warmup 2 >> gpurun_out/lm.log 2>&1 || exit 9
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_graph180 -o run -- python bench.py --steps 25 --warmup 5 --global-batch 180 --cuda-graph > gpurun_out/pgraph180.log 2>&1 || exit 10
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_charlm -o run -- python bench/lm_bench.py --config charlm --steps 3 --warmup 1 > gpurun_out/pcharlm.log 2>&1 || exit 11
