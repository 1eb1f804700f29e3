set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_persist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_persist_tests.log 2>&1
tail -2 gpurun_out/r2_persist_tests.log
timeout -k 10 120 python -u bench/persist_bench.py > gpurun_out/r2_pb.log 2>&1
tail -1 gpurun_out/r2_pb.log
