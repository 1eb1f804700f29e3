set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cc_gputests.log 2>&1 || { tail -40 gpurun_out/cc_gputests.log; exit 1; }
tail -1 gpurun_out/cc_gputests.log
timeout -k 10 180 python bench.py > gpurun_out/cc_bench.log 2>&1
tail -1 gpurun_out/cc_bench.log
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --global-batch 180 --steps 200 --warmup 20 > gpurun_out/cc_bench_forced180.log 2>&1
tail -1 gpurun_out/cc_bench_forced180.log
