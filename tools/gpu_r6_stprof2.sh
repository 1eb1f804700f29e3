#!/bin/bash
set -e
export TMPDIR=/tmp
out=gpurun_out/stp2
mkdir -p $out
root=$PWD
timeout -k 10 300 env PDRNN_SW_FENCE_AB=1 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread \
  -k "latency_regime or seq_in_wave_step_gradients_match_fp64 and (180 or 512)" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in "fence PDRNN_SW_FENCE_AB=1" "grid PDRNN_SW=1" "nogrid PDRNN_SW_STEP_GRID_AB=1" "sw2 PDRNN_SW=2"; do
  set -- $v
  export $2
  cd /tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$1 -o run -- python3 $root/bench.py --steps 20 --warmup 5 --global-batch 180 --epoch-sequences 864 > $root/$out/$1.log 2>&1
  cd $root
  find /tmp/prof_$1 -name '*kernel_stats.csv' -exec cp {} $out/$1_stats.csv \;
  echo "== $1"; python3 - $out/$1_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:3]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:8.2f}")
PY
  for B in 180 512; do
    E=$((B * 24 / 5))
    timeout -k 10 180 env PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s${B}_$1.log 2>&1 || { tail -20 $out/s${B}_$1.log; exit 1; }
    tail -1 $out/s${B}_$1.log | python tools/bench_line.py "B=$B synced-graph $1"
  done
  unset PDRNN_SW PDRNN_SW_STEP_GRID_AB PDRNN_SW_FENCE_AB
done
