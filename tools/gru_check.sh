set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "gru or GRU" > gpurun_out/gru_tests.log 2>&1
timeout -k 10 120 python bench.py --cell gru --steps 200 --warmup 20 > gpurun_out/g2_bench.log 2>&1
tail -2 gpurun_out/gru_tests.log; tail -1 gpurun_out/g2_bench.log
