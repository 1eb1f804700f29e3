# fp32 large-H path (lstm_large.hip F32 storage): numerics tests, then the
# motion model at H=128 fp32 through bench.py, and the fp32 char-LM shape
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_coverage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || { tail -60 gpurun_out/f32_tests.log; exit 1; }
tail -2 gpurun_out/f32_tests.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --hidden 128 > gpurun_out/f32_motion_h128.log 2>&1
tail -1 gpurun_out/f32_motion_h128.log | cut -c1-200
