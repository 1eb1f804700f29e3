#!/bin/bash
# char-LM step glue: tests, dispatch trace of one step, benches
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-lmglue}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_lstm_persist.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python tools/charlm_glue_trace.py > $out/charlm_glue.txt 2> $out/trace_err.log || { tail -20 $out/trace_err.log; exit 1; }
for i in 1 2; do
  timeout -k 10 400 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 > $out/charlm_$i.log 2>&1 || { tail -20 $out/charlm_$i.log; exit 1; }
  tail -1 $out/charlm_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('charlm', d['value'], d['ms_per_step'], d.get('persist_fallbacks'))"
done
