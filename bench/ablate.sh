#!/bin/bash
# Timing ablations of the small-H LSTM kernels (diagnostic; rebuilds the
# extension with -DPDRNN_ABLATE=bits in the box's scratch copy, prints the
# in-kernel cycle stamps at B=180 (one sequence per workgroup, = 8-GPU
# per-rank batch)).
out=${1:-gpurun_out/ablate.log}
: > $out
for bits in 0 1 2 4 8 16 3 32 64 128; do
  PDRNN_HIP_EXTRA_FLAGS="-DPDRNN_ABLATE=$bits" python -m pytorch_distributed_rnn_amd._build > /dev/null || exit 1
  echo "ablate=$bits" >> $out
  PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench/kernels.py --batches 180 2>&1 | grep stamps | tail -2 >> $out || exit 1
done
