set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gprof2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof2 -o run -- python3 bench.py --cell gru --steps 25 --warmup 5 > gpurun_out/gprof2_bench.log 2>&1
