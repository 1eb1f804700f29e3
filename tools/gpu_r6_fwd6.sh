#!/bin/bash
# headline kernel table and benches after restricting the vector x staging to two-sequence maps
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-fwd6}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_train.py -x -q -k "seq_in_wave or bf16 or headline" --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
for cfg in "2 fp32" "2 fp32" "1 fp32" "1 bf16"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --gpus 1 --steps 100 --warmup 20 --layers $1 --dtype $2 > $out/b_$1_$2.log 2>&1 || { tail -20 $out/b_$1_$2.log; exit 1; }
  tail -1 $out/b_$1_$2.log | python tools/bench_line.py "layers=$1 $2"
done
