# round-3 GPU check: fused-step numerics (incl. the deferred-dW backward),
# headline bench, kernel table of the headline step.
#   tools/r3_check.sh TAG [pytest selection...]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3}
shift || true
sel=${@:-tests/test_gpu_train.py}
timeout -k 10 900 python -u -m pytest $sel -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -60 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/${tag}_bench.log 2>&1 || { tail -30 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/${tag}_bench180.log 2>&1 || { tail -30 gpurun_out/${tag}_bench180.log; exit 1; }
tail -1 gpurun_out/${tag}_bench180.log
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/${tag}_b1440_kernel_stats.md > /dev/null
head -12 gpurun_out/${tag}_b1440_kernel_stats.md
python tools/prof_window.py "$db" --anchor lstm_small_fwd --last 50 --out gpurun_out/${tag}_b1440_window.md
