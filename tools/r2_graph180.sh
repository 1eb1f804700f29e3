# the 8-GPU per-rank step proxy: synced step (forced RCCL collective) at B=180, eager vs graph replay
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 0 1; do
  PDRNN_CUDA_GRAPH=$g PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --global-batch 180 --steps 300 --warmup 30 > gpurun_out/g180_g$g.log 2>&1
  echo "graph=$g $(tail -1 gpurun_out/g180_g$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
PDRNN_CUDA_GRAPH=1 PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_g180 -o run -- python3 bench.py --global-batch 180 --steps 50 --warmup 10 > gpurun_out/g180_prof.log 2>&1
db=$(find /tmp/prof_g180 -name '*.db' | head -1)
python tools/prof_seq.py "$db" lstm_small_step_gs_kernel 215 2 > gpurun_out/g180_seq.txt
python tools/prof_summary.py "$db" --out gpurun_out/g180_kernel_stats.md
cat gpurun_out/g180_seq.txt
