set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/r2l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2l_gputests.log 2>&1 || { tail -40 gpurun_out/r2l_gputests.log; exit 1; }
tail -1 gpurun_out/r2l_gputests.log
timeout -k 10 600 python bench/lm_bench.py --config bilstm --batch 4096 --steps 5 --warmup 2 > gpurun_out/r2l_bilstm_b4096.log 2>&1
tail -1 gpurun_out/r2l_bilstm_b4096.log | cut -c1-250
for b in 128 512; do
timeout -k 10 600 python bench/lm_bench.py --config charlm --batch $b --steps 10 --warmup 2 > gpurun_out/r2l_charlm_b$b.log 2>&1
tail -1 gpurun_out/r2l_charlm_b$b.log | cut -c1-250
done
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/r2l/bilstm -o run -- python3 $R/bench/lm_bench.py --config bilstm --batch 4096 --steps 2 --warmup 1 > $R/gpurun_out/r2l_bilstm_prof.log 2>&1
cd $R
python tools/prof_summary.py $(find /tmp/r2l/bilstm -name '*.db' | head -1) > gpurun_out/r2l_bilstm_kernels.md
head -24 gpurun_out/r2l_bilstm_kernels.md | cut -c1-160
