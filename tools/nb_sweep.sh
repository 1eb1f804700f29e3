# Sweep sequences-per-workgroup of the fused motion step (fwd nb x bwd nb) at a batch size
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${1:-1440}
for f in 1 2; do for b in 1 2 3; do
  PDRNN_LSTM_NB_FWD=$f PDRNN_LSTM_NB_BWD=$b timeout -k 10 120 python bench.py --global-batch $B --steps 100 --warmup 10 > gpurun_out/sweep_tmp.log 2>&1
  echo "B=$B nb_fwd=$f nb_bwd=$b $(tail -1 gpurun_out/sweep_tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/nb_sweep.log
done; done
