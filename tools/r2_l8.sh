set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for b in 180 360; do
  timeout -k 10 120 python bench.py --global-batch $b --steps 300 --warmup 30 > gpurun_out/l8.log 2>&1
  echo "B=$b default(one-launch L=4) $(tail -1 gpurun_out/l8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  PDRNN_LSTM_BWD_L=8 timeout -k 10 120 python bench.py --global-batch $b --steps 300 --warmup 30 > gpurun_out/l8.log 2>&1
  echo "B=$b two-launch L=8 $(tail -1 gpurun_out/l8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  PDRNN_STEP_ONE_LAUNCH=0 timeout -k 10 120 python bench.py --global-batch $b --steps 300 --warmup 30 > gpurun_out/l8.log 2>&1
  echo "B=$b two-launch L=4 $(tail -1 gpurun_out/l8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
