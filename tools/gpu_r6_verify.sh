#!/bin/bash
# round-6 verification: the GPU tests touched this round, then the per-rank benches
set -e
export TMPDIR=/tmp
tag=${1:-v6}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py tests/test_gpu_kernels.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py tests/test_gpu_lstm_pipeline.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv.log 2>&1 || { tail -20 $out/drv.log; exit 1; }
tail -1 $out/drv.log | python tools/bench_line.py "driver-style"
for B in 1440 720 360 180; do
  E=$((B * 24 / 5))
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E > $out/b$B.log 2>&1 || { tail -20 $out/b$B.log; exit 1; }
  tail -1 $out/b$B.log | python tools/bench_line.py "B=$B eager"
  [ $B = 1440 ] && continue
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s$B.log 2>&1 || { tail -20 $out/s$B.log; exit 1; }
  tail -1 $out/s$B.log | python tools/bench_line.py "B=$B synced-graph"
done
