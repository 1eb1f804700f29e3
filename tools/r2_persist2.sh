set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u bench/persist_bench.py > gpurun_out/r2_pb.log 2>&1
tail -1 gpurun_out/r2_pb.log
PDRNN_LSTM_PERSIST=0 timeout -k 10 120 python -u bench/persist_bench.py >> gpurun_out/r2_pb.log 2>&1
tail -1 gpurun_out/r2_pb.log
timeout -k 10 120 python -u bench/persist_bench.py --seq 64 >> gpurun_out/r2_pb.log 2>&1
tail -1 gpurun_out/r2_pb.log
