set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_coverage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_fwd_tests.log 2>&1 || { tail -30 gpurun_out/r2_fwd_tests.log; exit 1; }
tail -2 gpurun_out/r2_fwd_tests.log
for m in bc gs; do
  PDRNN_LSTM_FWD_MAP=$m timeout -k 10 120 python bench/stamps.py 180,1440 > gpurun_out/r2_stamps_$m.log 2>&1
  PDRNN_LSTM_FWD_MAP=$m timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/r2_bench_$m.log 2>&1
  PDRNN_LSTM_FWD_MAP=$m timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/r2_bench180_$m.log 2>&1
  echo "== $m"; grep "fwd(train)" gpurun_out/r2_stamps_$m.log | sort -u | head -4
  tail -1 gpurun_out/r2_bench_$m.log | cut -c1-200; tail -1 gpurun_out/r2_bench180_$m.log | cut -c1-200
done
