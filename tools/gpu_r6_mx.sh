#!/bin/bash
# the reference's metric through the CLI (matrix), config 5
# (bi-LSTM h4096 fp16) and config 4 (char-LM) at HEAD
set -e
export TMPDIR=/tmp
tag=${1:-mx6}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python bench/runner.py --gpus 1 --results gpurun_out/$tag/matrix.jsonl --timeout 240 > gpurun_out/$tag/runner.log 2>&1 || { tail -30 gpurun_out/$tag/runner.log; exit 1; }
python bench/report.py --ours gpurun_out/$tag/matrix.jsonl > gpurun_out/$tag/matrix.md 2>&1
head -16 gpurun_out/$tag/matrix.md
timeout -k 10 400 python bench/lm_bench.py --config bilstm --steps 6 --warmup 2 > gpurun_out/$tag/bilstm.log 2>&1 || { tail -20 gpurun_out/$tag/bilstm.log; exit 1; }
tail -1 gpurun_out/$tag/bilstm.log | cut -c1-300
timeout -k 10 400 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 > gpurun_out/$tag/charlm.log 2>&1 || { tail -20 gpurun_out/$tag/charlm.log; exit 1; }
tail -1 gpurun_out/$tag/charlm.log | cut -c1-300
