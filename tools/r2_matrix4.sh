# reference metric rerun after the epoch-statistics read-back fix + first-run epoch profile
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u bench/epoch_profile.py > gpurun_out/epoch_profile4.log 2>&1
grep "Training Duration" gpurun_out/epoch_profile4.log
rm -f gpurun_out/r2_matrix4_n1.jsonl
timeout -k 10 900 python bench/runner.py --gpus 1 --results gpurun_out/r2_matrix4_n1.jsonl > gpurun_out/r2_matrix4_n1.log 2>&1
python bench/report.py --ours gpurun_out/r2_matrix4_n1.jsonl --dedup > gpurun_out/r2_matrix4_n1.md 2>&1 || python bench/report.py --ours gpurun_out/r2_matrix4_n1.jsonl > gpurun_out/r2_matrix4_n1.md 2>&1
head -16 gpurun_out/r2_matrix4_n1.md
