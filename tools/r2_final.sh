# round-end style check: build check, smoke, full GPU suite, benches, kernel stats of the headline
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r2f}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -30 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gputests.log 2>&1 || { tail -40 gpurun_out/${tag}_gputests.log; exit 1; }
tail -1 gpurun_out/${tag}_gputests.log
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch 180 > gpurun_out/${tag}_bench180.log 2>&1
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --cell gru > gpurun_out/${tag}_bench_gru.log 2>&1
timeout -k 10 180 python bench.py > gpurun_out/${tag}_bench_default.log 2>&1
for f in bench bench180 bench_gru bench_default; do tail -1 gpurun_out/${tag}_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['steps'], d['warmup'], d['epoch_time_s'])"; done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/${tag}_prof.log 2>&1
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_summary.py "$db" --out gpurun_out/${tag}_b1440_kernel_stats.md
head -10 gpurun_out/${tag}_b1440_kernel_stats.md
