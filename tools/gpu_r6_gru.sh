#!/bin/bash
# GRU on the sequence-in-wave map: fp64 tests, then B=1440 and synced per-rank benches (sw vs gate-split)
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-gru}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v -k "gru" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
grep -c PASSED $out/tests.log
for sw in 1 0; do
  PDRNN_SW=$sw timeout -k 10 240 python bench.py --cell gru --gpus 1 --steps 100 --warmup 20 > $out/b1440_sw$sw.log 2>&1 || { tail -20 $out/b1440_sw$sw.log; exit 1; }
  tail -1 $out/b1440_sw$sw.log | python tools/bench_line.py "GRU B=1440 sw=$sw"
done
for B in 720 360 180; do
  E=$((B * 24 / 5))
  for sw in 1 0; do
    PDRNN_SW=$sw PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --cell gru --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s${B}_sw$sw.log 2>&1 || { tail -20 $out/s${B}_sw$sw.log; exit 1; }
    tail -1 $out/s${B}_sw$sw.log | python tools/bench_line.py "GRU B=$B synced-graph sw=$sw"
  done
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cell gru --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
