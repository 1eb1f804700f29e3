# the reference's benchmark matrix through the CLI on one GPU (bench/runner.py:
# batch {480, 960, 1440} x trainer {local, distributed, horovod}), reported
# with bench/report.py next to the reference's own result files
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-mx}
rm -f gpurun_out/${tag}_matrix.jsonl
timeout -k 10 900 python bench/runner.py --gpus 1 --results gpurun_out/${tag}_matrix.jsonl --timeout 240 > gpurun_out/${tag}_runner.log 2>&1 || { tail -30 gpurun_out/${tag}_runner.log; exit 1; }
python bench/report.py --ours gpurun_out/${tag}_matrix.jsonl > gpurun_out/${tag}_matrix.md 2>&1
cat gpurun_out/${tag}_matrix.md
