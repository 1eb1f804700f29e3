# Full GPU verification pass (run through gpurun): GPU test suite, smoke, headline bench,
# and the multi-GPU step's launch sequence on one GPU (PDRNN_FORCE_GRAD_SYNC=1 at the
# 8-GPU per-rank batch: inline RCCL all-reduce + flat Adam after the fused step).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_n1.log 2>&1 || exit 3
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 180 >> gpurun_out/bench_n1.log 2>&1 || exit 4
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 180 >> gpurun_out/bench_n1.log 2>&1 || exit 5
