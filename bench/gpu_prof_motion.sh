# rocprofv3 kernel stats of the headline motion step at the 1-GPU (B=1440) and
# 8-GPU per-rank (B=180) batch sizes, in-kernel stamps, and a bi-LSTM batch sweep.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m1440 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/pm1440.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m180 -o run -- python bench.py --steps 25 --warmup 5 --global-batch 180 > gpurun_out/pm180.log 2>&1 || exit 2
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/bench_b180.log 2>&1 || exit 3
PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench/kernels.py --batches 180,1440 > gpurun_out/kernels.log 2>&1 || exit 4
for b in 512 1024 2048 4096; do
  timeout -k 10 200 python bench/lm_bench.py --config bilstm --steps 3 --warmup 1 --batch $b >> gpurun_out/bil_batch.log 2>&1 || exit 5
done
