set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s5_gputests.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5_smoke.log 2>&1
timeout -k 10 180 python bench.py > gpurun_out/s5_bench_n1.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/s5_bench_n1_200.log 2>&1
tail -3 gpurun_out/s5_gputests.log; tail -1 gpurun_out/s5_bench_n1.log; tail -1 gpurun_out/s5_bench_n1_200.log
