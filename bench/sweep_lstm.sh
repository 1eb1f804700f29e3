#!/bin/bash
# Sweep fused small-H LSTM launch configs (split x sequences-per-WG) on one GPU.
set -e
out=${1:-gpurun_out/sweep.log}
for sb in 2 4; do
  for sf in 2 4 8; do
    for nb in 1 2; do
      PDRNN_TUNE=split_fwd=$sf,split_bwd=$sb,nb_fwd=$nb \
        timeout -k 10 120 python bench/kernels.py --batches 1440,720,360,180 | sed "s/^/sf=$sf sb=$sb nb=$nb /" >> $out
    done
  done
done
