set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/warm_driver_$i.log 2>&1
  tail -1 gpurun_out/warm_driver_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-style', d['value'], d['ms_per_step'], d['epoch_time_s'])"
done
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/warm_200.log 2>&1
tail -1 gpurun_out/warm_200.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('200 steps', d['value'], d['ms_per_step'], d['epoch_time_s'])"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --global-batch 180 > gpurun_out/warm_180.log 2>&1
tail -1 gpurun_out/warm_180.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B180 driver-style', d['value'], d['ms_per_step'])"
