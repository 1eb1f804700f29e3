set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
export PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1
for g in 0 1; do PDRNN_CUDA_GRAPH=$g timeout -k 10 120 python bench/host_overhead.py --global-batch 180 --steps 300 2>&1 | tail -1; done
PDRNN_CUDA_GRAPH=1 timeout -k 10 120 python bench/host_overhead.py --global-batch 180 --steps 300 --cprofile > gpurun_out/host_cprofile.txt 2>&1
head -60 gpurun_out/host_cprofile.txt
