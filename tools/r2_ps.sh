set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ps.py -x -v --timeout 150 --timeout-method thread -k device > gpurun_out/r2_ps.log 2>&1 || true
grep -v "^\s*$" gpurun_out/r2_ps.log | grep -iv "amdgpu.ids" | tail -80
