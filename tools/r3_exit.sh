# exit status of forced-collective runs (native communicator teardown at exit) + 180 bench
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 2 --warmup 1 --ddp > gpurun_out/r3x_charlm.log 2>&1
echo "charlm ddp exit=$?"
PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --global-batch 180 > gpurun_out/r3x_b180_forced.log 2>&1
echo "bench forced exit=$?"
for B in 180 1440; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/r3x_bench$B.log 2>&1
  tail -1 gpurun_out/r3x_bench$B.log | cut -c1-200
done
