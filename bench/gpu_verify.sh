# Full GPU verification pass (run through gpurun): GPU test suite, smoke, headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 120 python bench.py > gpurun_out/bench_n1.log 2>&1 || exit 3
timeout -k 10 120 python bench.py --steps 200 --warmup 20 >> gpurun_out/bench_n1.log 2>&1 || exit 4
