set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
PDRNN_PS_MODE=8 timeout -k 10 120 python -u bench/persist_bench.py --reps 1 > gpurun_out/r2_ps_stamps.log 2>&1
grep "ps-stamp fwd" gpurun_out/r2_ps_stamps.log | sed -n '20,30p'
PDRNN_PS_MODE=15 timeout -k 10 120 python -u bench/persist_bench.py --reps 1 > gpurun_out/r2_ps_stamps15.log 2>&1
grep "ps-stamp fwd" gpurun_out/r2_ps_stamps15.log | sed -n '20,30p'
