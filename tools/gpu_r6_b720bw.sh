#!/bin/bash
# BPTT map at B = 720: mode 2 (one sequence per layer wave) vs mode 3 (two), loop stamps and kernel times
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-b720bw}
mkdir -p $out
for bm in 2 3; do
  PDRNN_LSTM_STAMPS=1 PDRNN_TUNE=sw_bwd_mode=$bm timeout -k 10 120 python bench.py --steps 4 --warmup 2 --global-batch 720 --epoch-sequences 2880 > $out/st_$bm.log 2>&1 || { tail -20 $out/st_$bm.log; exit 1; }
  echo "bwd mode $bm"; grep "\[stamps\] bwd" $out/st_$bm.log | tail -1 | cut -c1-260
done
