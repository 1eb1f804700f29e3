# bucket all-reduces beside the persistent recurrences: the test, then the
# same test under a kernel trace -> timeline of the overlap
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread -k "persistent_recurrence" > gpurun_out/ovp_test.log 2>&1 || { tail -40 gpurun_out/ovp_test.log; exit 1; }
tail -1 gpurun_out/ovp_test.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_ovp -o run -- python3 -m pytest $GRAFT_REPO_ROOT/tests/test_gpu_comm.py -x -q -p no:cacheprovider -k persistent_recurrence > $GRAFT_REPO_ROOT/gpurun_out/ovp_prof.log 2>&1
cd $GRAFT_REPO_ROOT
db=$(find /tmp/prof_ovp -name '*.db' | head -1)
python tools/prof_overlap.py "$db" > gpurun_out/ovp_overlap.md
cat gpurun_out/ovp_overlap.md | head -40
