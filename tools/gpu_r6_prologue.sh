#!/bin/bash
# entry / loop / exit stamps of the sequence-in-wave kernels: the prologue's share
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-prologue}
mkdir -p $out
for cfg in "1440 2 fp32" "1440 1 fp32" "1440 1 bf16" "720 2 fp32"; do
  set -- $cfg
  PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 4 --warmup 2 --global-batch $1 --epoch-sequences $(($1 * 4)) --layers $2 --dtype $3 > $out/st_$1_$2_$3.log 2>&1 || { tail -20 $out/st_$1_$2_$3.log; exit 1; }
  echo "B=$1 layers=$2 $3"; grep "stamps" $out/st_$1_$2_$3.log | tail -2 | cut -c1-330
done
