#!/bin/bash
# single-process epoch graph + capture-failure fallbacks + round-6 tests, then benches
set -e
export TMPDIR=/tmp
tag=${1:-gr}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread \
  -k "single_process_epoch_graph or capture_failure or epoch_graph_replay or graph_replayed or fused_step_matches or seq_in_wave_step or headline" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for i in 1 2; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv$i.log 2>&1 || { tail -20 $out/drv$i.log; exit 1; }
  tail -1 $out/drv$i.log | python tools/bench_line.py "driver-style $i"
done
timeout -k 10 240 python bench.py --steps 100 --warmup 10 > $out/s100.log 2>&1 || { tail -20 $out/s100.log; exit 1; }
tail -1 $out/s100.log | python tools/bench_line.py "100 steps"
timeout -k 10 240 env PDRNN_CUDA_GRAPH=0 python bench.py --steps 100 --warmup 10 > $out/s100_eager.log 2>&1 || { tail -20 $out/s100_eager.log; exit 1; }
tail -1 $out/s100_eager.log | python tools/bench_line.py "100 steps eager"
