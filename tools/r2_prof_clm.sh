set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_clm2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clm2 -o run -- python bench/lm_bench.py --config charlm --steps 3 --warmup 1 > gpurun_out/pc2.log 2>&1 || exit 2
f=$(find gpurun_out/prof_clm2 -name "*results.db" | head -1)
python tools/prof_summary.py "$f" --out gpurun_out/r2_charlm_persist_kernel_stats.md
head -30 gpurun_out/r2_charlm_persist_kernel_stats.md
rm -rf gpurun_out/prof_clm2
