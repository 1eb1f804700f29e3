#!/bin/bash
# Host-runtime sanitizer runs on the CPU (SURVEY.md §5 "Race detection"): the
# native communicator (csrc/runtime/comm.cpp: watchdog thread, close()
# draining), the bucketed reducers (reducer.cpp) and the bindings built with
# -fsanitize=<flavour> by g++, driven by the gloo multi-process tests.
#   tools/sanitize_host.sh address,undefined [pytest args...]
#   tools/sanitize_host.sh thread [pytest args...]
# The HIP device code is not sanitized (no GPU sanitizer on this pool).
set -e
cd "$(dirname "$0")/.."
flav=${1:-address,undefined}
shift || true
export PDRNN_SANITIZE=$flav
so=$(python -c "from pytorch_distributed_rnn_amd import _build; print(_build.build())" | tail -1)
unset PDRNN_SANITIZE
export PDRNN_EXT_SO=$so
case $flav in
  thread) rt=$(gcc -print-file-name=libtsan.so)
          # (report_mutex_bugs=0: the interpreter's and torch's static
          # destructors unlock already-destroyed mutexes at exit; data races are
          # still reported.  die_after_fork=0: the gloo tests fork rank processes from a
          # multi-threaded interpreter; one OpenMP thread: libgomp is not
          # instrumented and its barriers read as races / stall the runtime)
          export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 report_signal_unsafe=0 die_after_fork=0 report_mutex_bugs=0 suppressions=$PWD/tools/tsan.supp"
          export OMP_NUM_THREADS=1 ;;
  *)      rt="$(gcc -print-file-name=libasan.so)"
          case $flav in *undefined*) rt="$rt:$(gcc -print-file-name=libubsan.so)";; esac
          # the interpreter and torch are not instrumented: leaks at exit are theirs
          export ASAN_OPTIONS="detect_leaks=0 verify_asan_link_order=0 halt_on_error=1 abort_on_error=1"
          export UBSAN_OPTIONS="print_stacktrace=1 halt_on_error=1" ;;
esac
export LD_PRELOAD="$rt${LD_PRELOAD:+:$LD_PRELOAD}"
tests=${@:-tests/test_distributed_cpu.py tests/test_env_faults_cpu.py tests/test_optim_flat_cpu.py}
python -m pytest -x -q -p no:cacheprovider $tests
