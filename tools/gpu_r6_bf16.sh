#!/bin/bash
# bf16 vs fp32 motion step at --layers 1 and 2: benches and kernel tables
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-bf16}
mkdir -p $out
for L in 1 2; do
  for dt in fp32 bf16; do
    timeout -k 10 240 python bench.py --gpus 1 --steps 100 --warmup 20 --layers $L --dtype $dt > $out/b_${L}_$dt.log 2>&1 || { tail -20 $out/b_${L}_$dt.log; exit 1; }
    tail -1 $out/b_${L}_$dt.log | python tools/bench_line.py "layers=$L $dt"
  done
done
for dt in fp32 bf16; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof_$dt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --layers 1 --dtype $dt > $GRAFT_REPO_ROOT/$out/prof_$dt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof_$dt.log; exit 1; }
  cd $GRAFT_REPO_ROOT
done
