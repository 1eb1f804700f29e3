# kernel-trace windows of the default bench (B=1440, last 50 steps) and of the
# 8-GPU per-rank synced step (B=180, epoch graph replay).
#   tools/gpu_windows.sh TAG      (ANCHOR: the kernel that opens a step)
set -e
export TMPDIR=/tmp
tag=${1:-win}
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_window.py "$db" --anchor ${ANCHOR:-lstm_sw_fwd} --last 50 --out gpurun_out/${tag}_b1440_window.md
cat gpurun_out/${tag}_b1440_window.md | head -30
# the 8-GPU per-rank step (B=180, synced, epoch graph replay): the last 50
# steps of the 100 timed ones (bench.py then runs 3 + 100 per-step-graph steps)
cd /tmp
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag}_s180 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --global-batch 180 --epoch-sequences 864 --cuda-graph > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_s180.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_${tag}_s180 -name '*.db' | head -1)
python tools/prof_window.py "$db" --anchor ${ANCHOR:-lstm_sw_fwd} --end-skip 103 --first 50 --out gpurun_out/${tag}_s180_window.md
cat gpurun_out/${tag}_s180_window.md | head -30
