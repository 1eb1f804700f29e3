set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_coverage.py tests/test_gpu_gru_large.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32b_tests.log 2>&1 || { tail -40 gpurun_out/f32b_tests.log; exit 1; }
tail -1 gpurun_out/f32b_tests.log
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 > gpurun_out/f32b_h128_hip.log 2>&1
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 --cell gru > gpurun_out/f32b_h128_gru.log 2>&1
PDRNN_KERNELS=torch timeout -k 10 180 python bench.py --steps 30 --warmup 5 --hidden 128 --cell gru > gpurun_out/f32b_h128_gru_miopen.log 2>&1
for f in h128_hip h128_gru h128_gru_miopen; do tail -1 gpurun_out/f32b_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_f32b -o run -- python3 bench.py --steps 10 --warmup 3 --hidden 128 > gpurun_out/f32b_prof.log 2>&1
db=$(find /tmp/prof_f32b -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/f32b_h128_kernel_stats.md
head -12 gpurun_out/f32b_h128_kernel_stats.md
