# in-kernel loop / entry / exit stamps of the fused step at several batches
#   tools/r3_stamps.sh TAG [BATCH...]
set -e
export TMPDIR=/tmp
tag=${1:-r3s}; shift || true
mkdir -p gpurun_out
for B in ${@:-1440 720 180}; do
  PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch $B > gpurun_out/${tag}_stamps$B.log 2>&1
  echo "B=$B"; grep stamps gpurun_out/${tag}_stamps$B.log | tail -2
done
