# in-tree GEMM: numerics vs fp32 torch, then throughput vs hipBLASLt
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r3gemm}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u bench/gemm_bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -30 gpurun_out/${tag}_bench.log; exit 1; }
cat gpurun_out/${tag}_bench.log
