#!/bin/bash
# fp32 H = 128 LSTM with the multi-GPU sync sequence forced at world 1: direct gradients on / off
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-h128ab}
mkdir -p $out
for v in 1 0 1 0; do
  PDRNN_TUNE=direct_grads=$v PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench.py --hidden 128 --steps 20 --warmup 5 > $out/s_$v.log 2>&1 || { tail -20 $out/s_$v.log; exit 1; }
  tail -1 $out/s_$v.log | python tools/bench_line.py "H=128 forced sync direct_grads=$v"
done
for v in 1 0; do
  cd /tmp && PDRNN_TUNE=direct_grads=$v PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --hidden 128 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$out/prof_$v.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
done
