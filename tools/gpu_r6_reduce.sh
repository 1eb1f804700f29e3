#!/bin/bash
# slab reduction geometry: tests, kernel table at B = 1440 and 180, benches
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-reduce}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof180 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --global-batch 180 --epoch-sequences 864 > $GRAFT_REPO_ROOT/$out/prof180.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof180.log; exit 1; }
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 100 --warmup 20 > $out/b1440_$i.log 2>&1 || { tail -20 $out/b1440_$i.log; exit 1; }
  tail -1 $out/b1440_$i.log | python tools/bench_line.py "B=1440 run $i"
done
