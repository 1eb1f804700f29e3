set -e
mkdir -p gpurun_out
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 1440 720; do
  timeout -k 10 120 $D/sw_probe $B 20 3 > gpurun_out/dwab_256_$B.log 2>&1
  timeout -k 10 120 $D/sw_probe_dw512 $B 20 3 > gpurun_out/dwab_512_$B.log 2>&1
done
grep -h "^mode\|^B=\|chunks" gpurun_out/dwab_*.log
