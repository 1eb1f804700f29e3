set -e
export TMPDIR=/tmp
for cfg in "0 4" "1 4" "2 3" "2 4"; do
  set -- $cfg
  PDRNN_PRIO=$1 PDRNN_PRIO_SHIFT=$2 PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch 1440 > gpurun_out/r3p_$1_$2.log 2>&1
  echo "== prio $1 shift $2"; grep -A4 "grid=720" gpurun_out/r3p_$1_$2.log | grep "loop=\|decile" | tail -2 | cut -c1-300
  PDRNN_PRIO=$1 PDRNN_PRIO_SHIFT=$2 timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/r3p_$1_$2_bench.log 2>&1
  tail -1 gpurun_out/r3p_$1_$2_bench.log | cut -c1-220
done
