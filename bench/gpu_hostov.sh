# Host-enqueue vs device time of the motion step, and the RCCL launch gaps of
# the multi-GPU step sequence at the 8-GPU per-rank batch (PDRNN_FORCE_GRAD_SYNC=1).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/hostov.log
timeout -k 10 120 python bench/host_overhead.py --global-batch 180 >> gpurun_out/hostov.log 2>&1 || exit 1
PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench/host_overhead.py --global-batch 180 >> gpurun_out/hostov.log 2>&1 || exit 2
NCCL_GRAPH_MIXING_SUPPORT=0 PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 120 python bench/host_overhead.py --global-batch 180 >> gpurun_out/hostov.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NCCL_GRAPH_MIXING_SUPPORT=0 PDRNN_FORCE_GRAD_SYNC=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sync180_nomix -o run -- python bench.py --steps 25 --warmup 5 --global-batch 180 > gpurun_out/psync180.log 2>&1 || exit 4
