set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_lstm_pipeline.py tests/test_gpu_lstm_large.py tests/test_gpu_coverage.py -x -q --timeout 200 --timeout-method thread -k "direct or pipeline or large or coverage" > gpurun_out/dg_tests.log 2>&1 || { tail -30 gpurun_out/dg_tests.log; exit 1; }
tail -1 gpurun_out/dg_tests.log
for cell in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 10 > gpurun_out/dg_h128_$cell.log 2>&1
  tail -1 gpurun_out/dg_h128_$cell.log | python tools/bench_line.py "H=128 fp32 $cell"
done
BENCH_ARGS="--warmup 10" bash tools/gpu_timeline.sh dg_tl
