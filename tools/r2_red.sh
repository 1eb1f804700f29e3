set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/red_tests.log 2>&1 || { tail -40 gpurun_out/red_tests.log; exit 1; }
tail -1 gpurun_out/red_tests.log
for B in 1440 180; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/red_b$B.log 2>&1
  tail -1 gpurun_out/red_b$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['ms_per_step'])"
done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_red -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/red_prof.log 2>&1
db=$(find /tmp/prof_red -name '*.db' | head -1)
python tools/prof_seq.py "$db" lstm_small_bwd_gs_kernel 40 1
