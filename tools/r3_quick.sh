# quick GPU loop: fused-step tests + bench at the 1/2/8-GPU per-rank batches + kernel window
#   tools/r3_quick.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for B in 1440 720 180; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/${tag}_bench$B.log 2>&1 || { tail -20 gpurun_out/${tag}_bench$B.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['ms_per_step'], d['epoch_time_s'])"
done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_window.py "$db" --anchor lstm_small_fwd --last 50 --out gpurun_out/${tag}_b1440_window.md
