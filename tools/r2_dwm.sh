# BPTT dW on MFMA: full GPU suite, then headline benches (+ stamps)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_coverage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dwm_gputests.log 2>&1 || { tail -60 gpurun_out/dwm_gputests.log; exit 1; }
tail -1 gpurun_out/dwm_gputests.log
timeout -k 10 120 python bench/stamps.py 180,1440 > gpurun_out/dwm_stamps.log 2>&1
grep -E "stamps" gpurun_out/dwm_stamps.log | sort -u | head -8
for B in 1440 720 360 180; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/dwm_b$B.log 2>&1
  tail -1 gpurun_out/dwm_b$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['ms_per_step'])"
done
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cell gru > gpurun_out/dwm_gru.log 2>&1
tail -1 gpurun_out/dwm_gru.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('GRU', d['value'], d['ms_per_step'])"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/dwm_driver.log 2>&1
tail -1 gpurun_out/dwm_driver.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-style', d['value'], d['ms_per_step'])"
