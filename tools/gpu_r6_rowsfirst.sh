#!/bin/bash
# fp32 hidden 128: the row recurrence's backward with the first step fused
# (no lstm_large_bwd_first launch): equality suites, timeline, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rowsfirst
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lstm_persist.py \
  tests/test_gpu_lstm_pipeline.py tests/test_gpu_gru_large.py tests/test_gpu_lstm_large.py tests/test_gpu_train.py \
  > gpurun_out/rowsfirst/tests.log 2>&1 || { tail -40 gpurun_out/rowsfirst/tests.log; exit 1; }
tail -1 gpurun_out/rowsfirst/tests.log
BENCH_ARGS="--warmup 10" bash tools/gpu_timeline.sh r6h128d || exit 1
grep "GPU kernel time" gpurun_out/r6h128d_0_timeline.md
for c in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $c --steps 20 --warmup 10 > gpurun_out/rowsfirst/h128_$c.log 2>&1 \
    || { tail -20 gpurun_out/rowsfirst/h128_$c.log; exit 1; }
  tail -1 gpurun_out/rowsfirst/h128_$c.log | cut -c1-200
done
