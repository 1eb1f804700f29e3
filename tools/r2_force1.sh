# experiment: one-launch step at any batch (grid = B, one slab row per sequence)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
PDRNN_STEP_ONE_LAUNCH=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f1_tests.log 2>&1 || { tail -40 gpurun_out/f1_tests.log; exit 1; }
tail -1 gpurun_out/f1_tests.log
for b in 1440 720; do
  for v in 1 2; do
    PDRNN_STEP_ONE_LAUNCH=$v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --global-batch $b > gpurun_out/f1_b${b}_v$v.log 2>&1
    echo "B=$b mode=$v $(tail -1 gpurun_out/f1_b${b}_v$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
PDRNN_STEP_ONE_LAUNCH=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/prof_f1 -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/f1_prof.log 2>&1
db=$(find /tmp/prof_f1 -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/f1_b1440_kernel_stats.md
head -6 gpurun_out/f1_b1440_kernel_stats.md
