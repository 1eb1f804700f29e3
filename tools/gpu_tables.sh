# kernel tables (rocprofv3 --kernel-trace) of the large-H workloads: the
# in-tree GEMM coverage check (no Cijk_* / ATen reduce / Cat kernels)
#   tools/gpu_tables.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-tbl}
run_prof() {  # name, command...
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_${tag}_${name} -o run -- "$@" > $GRAFT_REPO_ROOT/gpurun_out/${tag}_${name}.log 2>&1)
  local db=$(find /tmp/prof_${tag}_${name} -name '*.db' | head -1)
  python tools/prof_summary.py "$db" --top 80 --title "$name" --out gpurun_out/${tag}_${name}_kernel_stats.md > /dev/null
  echo "== $name: $(tail -1 gpurun_out/${tag}_${name}.log | cut -c1-160)"
  grep -c "Cijk\|reduce_kernel\|CatArray" gpurun_out/${tag}_${name}_kernel_stats.md || true
}
run_prof bilstm python3 $GRAFT_REPO_ROOT/bench/lm_bench.py --config bilstm --steps 2 --warmup 1
run_prof motion_h128 python3 $GRAFT_REPO_ROOT/bench.py --hidden 128 --steps 10 --warmup 5
run_prof gru_h128 python3 $GRAFT_REPO_ROOT/bench.py --hidden 128 --cell gru --steps 10 --warmup 5
# last: the char-LM run (its process segfaulted at exit under rocprofv3 while
# the persistent recurrence used cooperative launches, rounds 4 rd2/rd4)
run_prof charlm python3 $GRAFT_REPO_ROOT/bench/lm_bench.py --config charlm --steps 4 --warmup 2
