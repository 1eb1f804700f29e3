# ordered kernel list of one fp32 --hidden 128 training step (where the ATen glue sits)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-seq}
for cell in lstm gru; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_${tag}_$cell -o run -- python3 $GRAFT_REPO_ROOT/bench.py --hidden 128 --cell $cell --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_$cell.log 2>&1)
  db=$(find /tmp/prof_${tag}_$cell -name '*.db' | head -1)
  python tools/prof_window.py "$db" --anchor lstm_rows_f32_fwd --skip 20 --first 4 --sequence 2 --out gpurun_out/${tag}_${cell}_h128_sequence.md > /dev/null
  head -120 gpurun_out/${tag}_${cell}_h128_sequence.md
done
