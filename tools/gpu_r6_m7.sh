#!/bin/bash
# Mode-7 A/B (three sequences per layer wave): fp64 gradient tests, the new
# round-6 tests, then the bench under each forced map.
set -e
export TMPDIR=/tmp
tag=${1:-m7}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "seq_in_wave or descriptor_range or sort_limit or embedding" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
run() {  # label, env...
  local lab=$1; shift
  timeout -k 10 240 env "$@" python bench.py --steps 100 --warmup 10 > $out/$lab.log 2>&1 || { tail -20 $out/$lab.log; exit 1; }
  tail -1 $out/$lab.log | python tools/bench_line.py "$lab"
}
run base PDRNN_X=0
run bwd7 PDRNN_SW_BWD_MODE=7
run fwd7 PDRNN_SW_MODE=7 PDRNN_SW_BWD_MODE=3
run both7 PDRNN_SW_MODE=7 PDRNN_SW_BWD_MODE=7
run base2 PDRNN_X=0

timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv.log 2>&1 || { tail -20 $out/drv.log; exit 1; }
tail -1 $out/drv.log | python tools/bench_line.py "driver-style"
