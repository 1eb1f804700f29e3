set -e
mkdir -p gpurun_out
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 180 1440; do
  timeout -k 10 120 $D/sw_probe $B 20 2 6 > gpurun_out/halfk_full_$B.log 2>&1
  timeout -k 10 120 $D/sw_probe_halfk $B 20 2 6 > gpurun_out/halfk_half_$B.log 2>&1 || true
done
grep -h "^mode\|^B=" gpurun_out/halfk_*.log
