#!/bin/bash
# four-wave forward (mode 5) at B = 180 / 360 / 512: loop / prologue stamps and the separate-launch kernel time
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-fwd4}
mkdir -p $out
for B in 180 360 512; do
  PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 4 --warmup 2 --global-batch $B --epoch-sequences $((B * 4)) > $out/st$B.log 2>&1 || { tail -20 $out/st$B.log; exit 1; }
  echo "B=$B"; grep "\[stamps\] fwd" $out/st$B.log | tail -1 | cut -c1-250
done
cd /tmp && PDRNN_SW=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --global-batch 180 --epoch-sequences 864 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
