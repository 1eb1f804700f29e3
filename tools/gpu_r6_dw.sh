#!/bin/bash
# dW ring-depth / chunk-count A/B at the headline batch (bench, 100 steps)
set -e
export TMPDIR=/tmp
tag=${1:-dwab}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "headline_batch_gradients or deferred_dw_gradients" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cfg in "4 256" "5 256" "6 256" "3 256" "4 384" "5 384" "4 192" "6 256"; do
  set -- $cfg
  timeout -k 10 240 env PDRNN_DW_STAGES=$1 PDRNN_DW_CHUNKS=$2 python bench.py --steps 100 --warmup 10 > $out/r$1_c$2.log 2>&1 || { tail -20 $out/r$1_c$2.log; exit 1; }
  tail -1 $out/r$1_c$2.log | python tools/bench_line.py "stages $1 chunks $2"
done
