set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r2_pb_modes.log
for m in 0 1 2 3 4 5 7; do
  PDRNN_PS_MODE=$m timeout -k 10 120 python -u bench/persist_bench.py --reps 3 > gpurun_out/r2_pb_m.log 2>&1
  echo "mode $m $(tail -1 gpurun_out/r2_pb_m.log)" | tee -a gpurun_out/r2_pb_modes.log
done
