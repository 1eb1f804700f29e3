# char-LM step: kernel table + the dispatch sequence of one whole step
#   tools/gpu_lmseq.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-lmseq}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 $GRAFT_REPO_ROOT/bench/lm_bench.py --config charlm --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_charlm.log 2>&1)
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_summary.py "$db" --top 60 --title charlm --out gpurun_out/${tag}_kernel_stats.md > /dev/null
python tools/prof_seq.py "$db" emb_fwd16 3 1 > gpurun_out/${tag}_step_seq.txt || true
tail -1 gpurun_out/${tag}_charlm.log | cut -c1-200
