#!/bin/bash
# per-phase stamps of the four-wave forward (mode 5) at B = 97 / 180 / 360 / 512
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-phase}
mkdir -p $out
for B in 180 97 360 512; do
  E=$((B * 4))
  PDRNN_LSTM_STAMPS=1 PDRNN_TUNE=sw_phase=1 timeout -k 10 120 python bench.py --steps 4 --warmup 2 --global-batch $B --epoch-sequences $E > $out/ph$B.log 2>&1 || { tail -20 $out/ph$B.log; exit 1; }
  echo "B=$B"; grep "phases\|fwd(head" $out/ph$B.log | tail -3
done
