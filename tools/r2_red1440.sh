set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rd_tests.log 2>&1 || { tail -40 gpurun_out/rd_tests.log; exit 1; }
tail -1 gpurun_out/rd_tests.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/rd_b1440.log 2>&1
  echo "B=1440 $(tail -1 gpurun_out/rd_b1440.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch 720 > gpurun_out/rd_b720.log 2>&1
  echo "B=720 $(tail -1 gpurun_out/rd_b720.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/prof_rd -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/rd_prof.log 2>&1
db=$(find /tmp/prof_rd -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/rd_b1440_kernel_stats.md
grep slab_reduce gpurun_out/rd_b1440_kernel_stats.md
