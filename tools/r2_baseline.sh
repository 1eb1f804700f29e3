set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/r2_bench_n1.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/r2_bench_b180.log 2>&1
tail -3 gpurun_out/r2_gputests.log; tail -1 gpurun_out/r2_bench_n1.log; tail -1 gpurun_out/r2_bench_b180.log
