set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c1_gputests.log 2>&1
timeout -k 10 120 python bench.py --cell gru --steps 200 --warmup 20 > gpurun_out/c1_bench_gru.log 2>&1
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/c1_bench.log 2>&1
tail -1 gpurun_out/c1_gputests.log; tail -1 gpurun_out/c1_bench_gru.log; tail -1 gpurun_out/c1_bench.log
