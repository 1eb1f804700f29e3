set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_comm_tests.log 2>&1
cd /tmp
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r2_commtrace -o run -- python3 $GRAFT_REPO_ROOT/bench/comm_trace.py > $GRAFT_REPO_ROOT/gpurun_out/r2_commtrace.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find gpurun_out/r2_commtrace -name '*.db' | head -1)
python tools/prof_streams.py $db --out gpurun_out/r2_commtrace_streams.md > /dev/null
tail -5 gpurun_out/r2_comm_tests.log; head -30 gpurun_out/r2_commtrace_streams.md
