# round check: every GPU test, smoke(), the default bench and the B=180 bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3f}
timeout -k 10 1500 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/${tag}_bench180.log 2>&1 || { tail -20 gpurun_out/${tag}_bench180.log; exit 1; }
tail -1 gpurun_out/${tag}_bench180.log | cut -c1-300
