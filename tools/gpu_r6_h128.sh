#!/bin/bash
# fp32 H = 128: GPU tests of the DDP / pipeline paths with direct gradients, then benches (plain and
# with the multi-GPU sync sequence forced at world 1)
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-h128}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_lstm_pipeline.py tests/test_gpu_gru_large.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for c in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $c --steps 20 --warmup 5 > $out/h128_$c.log 2>&1 || { tail -20 $out/h128_$c.log; exit 1; }
  tail -1 $out/h128_$c.log | python tools/bench_line.py "H=128 $c"
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --hidden 128 --cell $c --steps 20 --warmup 5 > $out/h128s_$c.log 2>&1 || { tail -20 $out/h128s_$c.log; exit 1; }
  tail -1 $out/h128s_$c.log | python tools/bench_line.py "H=128 $c forced sync"
done
