# reference metric (1-epoch CLI, rank-0 Training Duration) at 1 GPU + bf16 1-layer config 2
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r2_matrix2_n1.jsonl
timeout -k 10 900 python bench/runner.py --gpus 1 --results gpurun_out/r2_matrix2_n1.jsonl > gpurun_out/r2_matrix2_n1.log 2>&1
grep -c returncode gpurun_out/r2_matrix2_n1.jsonl
python bench/report.py --ours gpurun_out/r2_matrix2_n1.jsonl --dedup > gpurun_out/r2_matrix2_n1.md 2>&1 || python bench/report.py --ours gpurun_out/r2_matrix2_n1.jsonl > gpurun_out/r2_matrix2_n1.md 2>&1
head -30 gpurun_out/r2_matrix2_n1.md
timeout -k 10 180 python bench.py --dtype bf16 --layers 1 --steps 200 --warmup 20 > gpurun_out/r2_bf16_1l.log 2>&1
tail -1 gpurun_out/r2_bf16_1l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bf16 1x32', d['value'], d['ms_per_step'])"
