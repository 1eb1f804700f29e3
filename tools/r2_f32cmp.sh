# fp32 H=128 motion model: HIP large-H kernels vs the stock MIOpen path, + kernel stats
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 > gpurun_out/f32_h128_hip.log 2>&1
PDRNN_KERNELS=torch timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 > gpurun_out/f32_h128_miopen.log 2>&1
for f in hip miopen; do tail -1 gpurun_out/f32_h128_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_f32 -o run -- python3 bench.py --steps 10 --warmup 3 --hidden 128 > gpurun_out/f32_prof.log 2>&1
db=$(find /tmp/prof_f32 -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/f32_h128_kernel_stats.md
head -16 gpurun_out/f32_h128_kernel_stats.md
