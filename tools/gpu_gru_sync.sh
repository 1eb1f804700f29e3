set -e
mkdir -p gpurun_out
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --cell gru --steps 200 --warmup 20 --global-batch 180 --epoch-sequences 864 --cuda-graph > gpurun_out/r5g_synced180_gru.log 2>&1
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 PDRNN_CUDA_GRAPH=0 timeout -k 10 180 python bench.py --cell gru --steps 200 --warmup 20 --global-batch 180 --epoch-sequences 864 > gpurun_out/r5g_synced180_gru_eager.log 2>&1
tail -1 gpurun_out/r5g_synced180_gru.log | python tools/bench_line.py "GRU B=180 synced graph"
tail -1 gpurun_out/r5g_synced180_gru_eager.log | python tools/bench_line.py "GRU B=180 synced eager"
