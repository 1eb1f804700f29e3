set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for v in 0 1; do
  PDRNN_BF16_WROUND=$v timeout -k 10 120 python bench.py --layers 1 --dtype bf16 --steps 300 --warmup 30 > gpurun_out/bfab.log 2>&1
  echo "1x32 bf16 wround=$v $(tail -1 gpurun_out/bfab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  PDRNN_BF16_WROUND=$v timeout -k 10 120 python bench.py --dtype bf16 --steps 300 --warmup 30 --global-batch 180 > gpurun_out/bfab.log 2>&1
  echo "2x32 bf16 B=180 wround=$v $(tail -1 gpurun_out/bfab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 120 python bench.py --layers 1 --steps 300 --warmup 30 > gpurun_out/bfab.log 2>&1
echo "1x32 fp32 $(tail -1 gpurun_out/bfab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
