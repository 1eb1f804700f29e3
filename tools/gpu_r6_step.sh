#!/bin/bash
# one-launch latency-regime step: tests, then separate (PDRNN_SW=2) vs one-launch benches
set -e
export TMPDIR=/tmp
tag=${1:-st}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread \
  -k "seq_in_wave or sw_step or latency_regime or single_process or capture_failure or epoch_graph_replay or graph_replayed or fused_step_matches or one_launch" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for B in 180 360 512; do
  E=$((B * 24 / 5))
  for sw in 2 1; do
    timeout -k 10 180 env PDRNN_SW=$sw python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E > $out/b${B}_sw$sw.log 2>&1 || { tail -20 $out/b${B}_sw$sw.log; exit 1; }
    tail -1 $out/b${B}_sw$sw.log | python tools/bench_line.py "B=$B eager PDRNN_SW=$sw"
    timeout -k 10 180 env PDRNN_SW=$sw PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s${B}_sw$sw.log 2>&1 || { tail -20 $out/s${B}_sw$sw.log; exit 1; }
    tail -1 $out/s${B}_sw$sw.log | python tools/bench_line.py "B=$B synced-graph PDRNN_SW=$sw"
  done
done
