# kernel sequence + stats of the per-rank step at the 8-GPU per-rank batch (B=180)
timeout -k 10 400 python -u -m pytest tests/test_gpu_ps.py -x -v --timeout 150 --timeout-method thread > gpurun_out/ps_gpu.log 2>&1 || { tail -40 gpurun_out/ps_gpu.log; exit 1; }; tail -3 gpurun_out/ps_gpu.log
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_s180 -o run -- python3 bench.py --steps 50 --warmup 10 --global-batch 180 > gpurun_out/s180_prof.log 2>&1
db=$(find /tmp/prof_s180 -name '*.db' | head -1)
python tools/prof_seq.py "$db" lstm_small_bwd_gs_kernel 210 2 > gpurun_out/s180_seq.txt
python tools/prof_summary.py "$db" --out gpurun_out/s180_kernel_stats.md
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_s180s -o run -- python3 bench.py --steps 50 --warmup 10 --global-batch 180 > gpurun_out/s180s_prof.log 2>&1
db=$(find /tmp/prof_s180s -name '*.db' | head -1)
python tools/prof_seq.py "$db" lstm_small_bwd_gs_kernel 210 2 > gpurun_out/s180s_seq.txt
python tools/prof_summary.py "$db" --out gpurun_out/s180s_kernel_stats.md
tail -1 gpurun_out/s180_prof.log; tail -1 gpurun_out/s180s_prof.log
cat gpurun_out/s180_seq.txt gpurun_out/s180s_seq.txt
