# one PMC pass over the persistent-kernel layer bench; the profiled process
# segfaults in its exit path after the CSV is written (same with --kernel-trace),
# so each pass is its own call and nothing runs after it
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d $R/gpurun_out/pmcp/$2 -o run -- python3 $R/bench/persist_bench.py --reps 1 --seq 128 > $R/gpurun_out/pmcp/$2.log 2>&1
