#!/bin/bash
# vector x staging: fp64 tests of every sw map (fp32 and bf16 inputs), prologue stamps, benches
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-xstage}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q -k "seq_in_wave or headline_batch or one_launch or bf16 or fused" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cfg in "1440 2 fp32" "1440 1 fp32" "1440 1 bf16" "180 2 fp32" "720 2 fp32"; do
  set -- $cfg
  PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 4 --warmup 2 --global-batch $1 --epoch-sequences $(($1 * 4)) --layers $2 --dtype $3 > $out/st_$1_$2_$3.log 2>&1 || { tail -20 $out/st_$1_$2_$3.log; exit 1; }
  echo "B=$1 layers=$2 $3"; grep "\[stamps\] fwd" $out/st_$1_$2_$3.log | tail -1 | cut -c1-200
done
for L in 1 2; do
  for dt in fp32 bf16; do
    timeout -k 10 240 python bench.py --gpus 1 --steps 100 --warmup 20 --layers $L --dtype $dt > $out/b_${L}_$dt.log 2>&1 || { tail -20 $out/b_${L}_$dt.log; exit 1; }
    tail -1 $out/b_${L}_$dt.log | python tools/bench_line.py "layers=$L $dt"
  done
done
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv.log 2>&1 || { tail -20 $out/drv.log; exit 1; }
tail -1 $out/drv.log | python tools/bench_line.py "driver-style"
for B in 720 360 180; do
  E=$((B * 24 / 5))
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s$B.log 2>&1 || { tail -20 $out/s$B.log; exit 1; }
  tail -1 $out/s$B.log | python tools/bench_line.py "B=$B synced-graph"
done
