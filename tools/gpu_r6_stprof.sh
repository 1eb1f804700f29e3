#!/bin/bash
# one-launch latency step: quick tests, then kernel stats (B=180) of the three forms
set -e
export TMPDIR=/tmp
out=gpurun_out/stp
mkdir -p $out
root=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread \
  -k "seq_in_wave or sw_step or latency_regime or single_process or fused_step_matches" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in "sw2 PDRNN_SW=2" "grid PDRNN_SW=1" "nogrid PDRNN_SW_STEP_GRID_AB=1"; do
  set -- $v
  export $2
  cd /tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$1 -o run -- python3 $root/bench.py --steps 20 --warmup 5 --global-batch 180 --epoch-sequences 864 > $root/$out/$1.log 2>&1
  cd $root
  find /tmp/prof_$1 -name '*kernel_stats.csv' -exec cp {} $out/$1_stats.csv \;
  unset PDRNN_SW PDRNN_SW_STEP_GRID_AB
  echo "== $1"; python3 - $out/$1_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:5]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:8.2f}")
PY
done
for B in 180 360 512; do
  E=$((B * 24 / 5))
  for sw in 2 1; do
    timeout -k 10 180 env PDRNN_SW=$sw python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E > $out/b${B}_sw$sw.log 2>&1 || { tail -20 $out/b${B}_sw$sw.log; exit 1; }
    tail -1 $out/b${B}_sw$sw.log | python tools/bench_line.py "B=$B eager PDRNN_SW=$sw"
    timeout -k 10 180 env PDRNN_SW=$sw PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > $out/s${B}_sw$sw.log 2>&1 || { tail -20 $out/s${B}_sw$sw.log; exit 1; }
    tail -1 $out/s${B}_sw$sw.log | python tools/bench_line.py "B=$B synced-graph PDRNN_SW=$sw"
  done
done
