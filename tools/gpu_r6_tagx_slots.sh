#!/bin/bash
# Tagged exchange ring length: does re-reading the same slot lines (2-slot
# ring) cost the polls stale-line latency?  slots=512 = a fresh slot a step.
set -o pipefail
mkdir -p gpurun_out/tagx
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lstm_persist.py \
  -k tagged > gpurun_out/tagx/tests_slots.log 2>&1 || { tail -30 gpurun_out/tagx/tests_slots.log; exit 1; }
tail -1 gpurun_out/tagx/tests_slots.log
for v in persist_tagx=0 persist_tagx=1,persist_tagx_slots=2 persist_tagx=1,persist_tagx_slots=8 persist_tagx=1,persist_tagx_slots=512; do
  PDRNN_TUNE=$v,persist_stamps=1 timeout -k 10 240 python bench/lm_bench.py --config charlm --steps 2 --warmup 1 \
    > gpurun_out/tagx/st_$v.log 2>&1 || { tail -20 gpurun_out/tagx/st_$v.log; exit 1; }
  echo "$v:"; grep "persist stamps] fwd" gpurun_out/tagx/st_$v.log | tail -1
done
