# full GPU test suite + N=1 benches (LSTM B=1440 / B=180, GRU) + loop stamps
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gputests.log 2>&1 || { tail -40 gpurun_out/${tag}_gputests.log; exit 1; }
tail -2 gpurun_out/${tag}_gputests.log
timeout -k 10 120 python bench/stamps.py 180,1440 > gpurun_out/${tag}_stamps.log 2>&1
grep -E "stamps" gpurun_out/${tag}_stamps.log | sort -u | head -8
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/${tag}_bench180.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --cell gru > gpurun_out/${tag}_bench_gru.log 2>&1
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_driver.log 2>&1
for f in bench bench180 bench_gru bench_driver; do tail -1 gpurun_out/${tag}_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['config']['model'])"; done
