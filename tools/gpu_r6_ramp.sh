#!/bin/bash
# Short-window overhead probe: the driver's bench line under warm-up variants.
set -e
export TMPDIR=/tmp
tag=${1:-r6ramp}
out=gpurun_out/$tag
mkdir -p $out
run() {  # label, env..., -- bench args
  local lab=$1; shift
  timeout -k 10 240 env "$@" > $out/$lab.log 2>&1 || { tail -20 $out/$lab.log; exit 1; }
  tail -1 $out/$lab.log | python tools/bench_line.py "$lab"
}
run d1 python bench.py --steps 20 --warmup 5
run d2 python bench.py --steps 20 --warmup 5
run w300 PDRNN_WARMUP_MS=300 python bench.py --steps 20 --warmup 5
run w300b PDRNN_WARMUP_MS=300 python bench.py --steps 20 --warmup 5
run w50 python bench.py --steps 20 --warmup 50
run s100 python bench.py --steps 100 --warmup 5
run s20w5_gr PDRNN_CUDA_GRAPH=1 python bench.py --steps 20 --warmup 5
