#!/bin/bash
# full GPU suite (as the driver runs it), smoke(), the default bench and a kernel table of the headline step
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-full}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
tail -1 $out/bench_default.log
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
