# kernel-trace window of the 2-GPU per-rank synced step (B=720, epoch graph)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_w720 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --global-batch 720 --epoch-sequences 3456 --cuda-graph > $GRAFT_REPO_ROOT/gpurun_out/w720_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_w720 -name '*.db' | head -1)
python tools/prof_window.py "$db" --anchor lstm_sw_fwd --end-skip 103 --first 50 --out gpurun_out/w720_window.md
head -14 gpurun_out/w720_window.md
