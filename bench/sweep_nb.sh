#!/bin/bash
# Sweep sequences-per-workgroup (nb) of the fused forward / backward on bench.py.
set -e
out=${1:-gpurun_out/sweep_nb.log}
: > $out
for nbf in 1 2; do
  for nbb in 1 2 3; do
    echo "nb_fwd=$nbf nb_bwd=$nbb" >> $out
    PDRNN_TUNE=nb_fwd=$nbf,nb_bwd=$nbb timeout -k 10 120 python bench.py --steps 50 --warmup 10 2>/dev/null | tail -1 >> $out
  done
done
