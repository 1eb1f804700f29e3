# N=1 CLI matrix (Training Duration = the reference metric) at 480/960/1440
# for local/distributed/horovod, next to bench.py's epoch_time_s at the same batches
set -e
export TMPDIR=/tmp
tag=${1:-r3mx}
mkdir -p gpurun_out
rm -f gpurun_out/${tag}.jsonl
timeout -k 10 900 python bench/runner.py --results gpurun_out/${tag}.jsonl --gpus 1 --batches 480 960 1440 --timeout 240 > gpurun_out/${tag}_runner.log 2>&1
python bench/report.py --ours gpurun_out/${tag}.jsonl > gpurun_out/${tag}.md 2>&1
for B in 480 960 1440; do
  timeout -k 10 180 python bench.py --steps 100 --warmup 20 --global-batch $B > gpurun_out/${tag}_bench$B.log 2>&1
  tail -1 gpurun_out/${tag}_bench$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench B=$B epoch_time_s', d['epoch_time_s'], 'ms/step', d['ms_per_step'])" >> gpurun_out/${tag}.md
done
cat gpurun_out/${tag}.md
