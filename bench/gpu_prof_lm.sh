# rocprofv3 kernel stats of the secondary benchmarks (char-LM h1024, bi-LSTM h4096 B=4096).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bil -o run -- python bench/lm_bench.py --config bilstm --steps 2 --warmup 1 > gpurun_out/pb.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clm -o run -- python bench/lm_bench.py --config charlm --steps 2 --warmup 1 > gpurun_out/pc.log 2>&1 || exit 2
