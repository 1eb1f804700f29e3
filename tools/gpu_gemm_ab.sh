# fp32 GEMM change check: GEMM numerics tests, the dW probe, the fp32 H=128 benches
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-gab}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_lstm_pipeline.py tests/test_gpu_lstm_large.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 120 python bench/gemm_f32_probe.py | tail -1
NO_TESTS=1 bash tools/gpu_pipe.sh ${tag}l
NO_TESTS=1 CELL=gru bash tools/gpu_pipe.sh ${tag}g
