# one GPU round trip: motion fused-step tests + A/B of the own-tile dW backward,
# stamps and a kernel-trace window; then the GEMM / large-H tests and LM benches
#   tools/gpu_fused.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-fz}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for f in 0 1; do
  PDRNN_BWD_DW_FUSED=$f timeout -k 10 180 python bench.py > gpurun_out/${tag}_bench_fused$f.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_fused$f.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench_fused$f.log | python tools/bench_line.py "fused=$f"
done
PDRNN_LSTM_STAMPS=1 timeout -k 10 180 python bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_stamps.log 2>&1 || { tail -20 gpurun_out/${tag}_stamps.log; exit 1; }
grep "stamps\] bwd" gpurun_out/${tag}_stamps.log | tail -2
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_${tag} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_${tag} -name '*.db' | head -1)
python tools/prof_window.py "$db" --anchor lstm_small_fwd --last 50 --out gpurun_out/${tag}_b1440_window.md
head -12 gpurun_out/${tag}_b1440_window.md
bash tools/gpu_lm.sh ${tag}lm
