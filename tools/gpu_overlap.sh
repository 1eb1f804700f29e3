# bwd || dW overlap probe at the 1/2-GPU per-rank batches
set -e
mkdir -p gpurun_out
P=pytorch_distributed_rnn_amd/build_native/probe/sw_probe
for B in 1440 720; do PROBE_OVERLAP=1 timeout -k 10 120 $P $B 20 3 2 >> gpurun_out/overlap_probe.log 2>&1; done
