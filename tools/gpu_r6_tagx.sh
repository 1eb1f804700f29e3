#!/bin/bash
# Tagged h exchange of the persistent forward (PDRNN_TUNE persist_tagx):
# equality tests, then the char-LM bench A/B and the per-step phase stamps.
set -o pipefail
mkdir -p gpurun_out/tagx
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lstm_persist.py \
  > gpurun_out/tagx/tests.log 2>&1 || { tail -30 gpurun_out/tagx/tests.log; exit 1; }
tail -3 gpurun_out/tagx/tests.log
for v in 0 1 0 1; do
  PDRNN_TUNE=persist_tagx=$v timeout -k 10 240 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 \
    > gpurun_out/tagx/bench_$v.log 2>&1 || { tail -20 gpurun_out/tagx/bench_$v.log; exit 1; }
  echo "tagx=$v: $(tail -1 gpurun_out/tagx/bench_$v.log)"
done
for v in 1; do
  PDRNN_TUNE=persist_tagx=$v,persist_stamps=1 timeout -k 10 240 python bench/lm_bench.py --config charlm --steps 2 --warmup 1 \
    > gpurun_out/tagx/stamps_$v.log 2>&1 || { tail -20 gpurun_out/tagx/stamps_$v.log; exit 1; }
  echo "tagx=$v:"; grep "persist stamps" gpurun_out/tagx/stamps_$v.log | tail -2
done
