#!/bin/bash
# round-6 HEAD numbers: every headline / config bench in one call (jsonl + summary lines)
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-head}
mkdir -p $out
: > $out/lines.jsonl
b() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  tail -1 $out/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['name']='$name'; print(json.dumps(d))" >> $out/lines.jsonl
  tail -1 $out/lines.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['name'], d['value'], d['unit'], d['ms_per_step'])"
}
b headline_default 300 python bench.py
b headline_100 300 python bench.py --steps 100 --warmup 20
b driver_20_5 300 python bench.py --gpus 1 --steps 20 --warmup 5
b layers1_fp32 300 python bench.py --steps 100 --warmup 20 --layers 1
b layers1_bf16 300 python bench.py --steps 100 --warmup 20 --layers 1 --dtype bf16
b layers2_bf16 300 python bench.py --steps 100 --warmup 20 --dtype bf16
b gru 300 python bench.py --steps 100 --warmup 20 --cell gru
for B in 720 360 180; do
  E=$((B * 24 / 5))
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 b synced_$B 240 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 b synced_gru_$B 240 python bench.py --cell gru --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph
done
b h128_lstm 300 python bench.py --hidden 128 --steps 20 --warmup 5
b h128_gru 300 python bench.py --hidden 128 --cell gru --steps 20 --warmup 5
b charlm 400 python bench/lm_bench.py --config charlm --steps 10 --warmup 3
b bilstm 900 python bench/lm_bench.py --config bilstm --steps 4 --warmup 2
