# Two ranks on the box's single GPU: (a) gloo backend with the fused GPU step
# (exercises the world>1 step: ProcessGroupComm all-reduce + flat Adam),
# (b) RCCL backend (RCCL may refuse two ranks on one device: logged, not fatal).
set -o pipefail
mkdir -p gpurun_out
PDRNN_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/b2_gloo.log 2>&1 || exit 1
NCCL_DEBUG=WARN timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/b2_rccl.log 2>&1
echo "rccl 2-rank exit: $?" >> gpurun_out/b2_rccl.log
exit 0
