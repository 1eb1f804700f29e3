# (1) reference result matrix at 1 GPU through the real CLI, (2) char-LM DDP
# overlap trace + forced-collective cost, (3) bi-LSTM h4096 sized to HBM
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out /tmp/r2prof
timeout -k 10 900 python bench/runner.py --gpus 1 --results gpurun_out/r2_matrix_n1.jsonl > gpurun_out/r2_matrix_n1.log 2>&1
grep -c returncode gpurun_out/r2_matrix_n1.jsonl
timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 2 > gpurun_out/r2_charlm_plain.log 2>&1
PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 2 --ddp > gpurun_out/r2_charlm_ddp.log 2>&1
tail -1 gpurun_out/r2_charlm_plain.log | cut -c1-220; tail -1 gpurun_out/r2_charlm_ddp.log | cut -c1-220
cd /tmp
PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r2prof/charlm -o run -- python3 $R/bench/lm_bench.py --config charlm --steps 2 --warmup 1 --ddp > $R/gpurun_out/r2_charlm_trace.log 2>&1
cd $R
db=$(find /tmp/r2prof/charlm -name '*.db' | head -1)
python tools/prof_streams.py $db --out gpurun_out/r2_charlm_overlap.md > /dev/null
python tools/prof_summary.py $db > gpurun_out/r2_charlm_kernels.md
head -30 gpurun_out/r2_charlm_overlap.md
timeout -k 10 600 python bench/lm_bench.py --config bilstm --batch 8192 --steps 3 --warmup 1 > gpurun_out/r2_bilstm_b8192.log 2>&1
tail -1 gpurun_out/r2_bilstm_b8192.log | cut -c1-400
