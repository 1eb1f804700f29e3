set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gprof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o run -- python3 bench.py --cell gru --steps 25 --warmup 5 > gpurun_out/gprof_bench.log 2>&1
timeout -k 10 120 python bench.py --cell gru --steps 200 --warmup 20 > gpurun_out/g_bench.log 2>&1
PDRNN_LSTM_NB_FWD=2 timeout -k 10 120 python bench.py --cell gru --steps 200 --warmup 20 > gpurun_out/g_bench_nb2.log 2>&1 || true
tail -1 gpurun_out/g_bench.log; tail -2 gpurun_out/g_bench_nb2.log
