#!/bin/bash
# forward map A/B at the 2-GPU per-rank batch (B = 720) and 1024: mode 2 (default) vs mode 5, synced epoch graph
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-m5ab}
mkdir -p $out
for B in 720 1024; do
  E=$((B * 24 / 5))
  for fm in 2 5 2 5; do
    PDRNN_TUNE=sw_mode=$fm,sw_bwd_mode=2 PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s${B}_$fm.log 2>&1 || { tail -20 $out/s${B}_$fm.log; exit 1; }
    tail -1 $out/s${B}_$fm.log | python tools/bench_line.py "B=$B fwd mode $fm"
  done
done
