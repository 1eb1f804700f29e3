set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_lstm_large.py -x -q > gpurun_out/tl.log 2>&1 || exit 1
timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 5 --warmup 2 > gpurun_out/lm_charlm.log 2>&1 || exit 2
timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 3 --warmup 1 > gpurun_out/lm_bilstm.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bil -o run -- python bench/lm_bench.py --config bilstm --steps 2 --warmup 1 > gpurun_out/pb.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clm -o run -- python bench/lm_bench.py --config charlm --steps 2 --warmup 1 > gpurun_out/pc.log 2>&1 || exit 6
