# fp32 dW GEMM shape of the motion --hidden-units 128 model: wall time and PMC
# passes (FETCH_SIZE; MFMA / LDS-wait cycles) -> gpurun_out/probe_pmc.md
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python bench/gemm_f32_probe.py $PROBE_ARGS > gpurun_out/probe_time.log 2>&1; tail -1 gpurun_out/probe_time.log
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench/gemm_f32_probe.py --iters 5 $PROBE_ARGS > $GRAFT_REPO_ROOT/gpurun_out/probe_pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d /tmp/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/bench/gemm_f32_probe.py --iters 5 $PROBE_ARGS > $GRAFT_REPO_ROOT/gpurun_out/probe_pmc2.log 2>&1
cd $GRAFT_REPO_ROOT
python tools/pmc_summary.py gpurun_out/probe_pmc.md /tmp/pmc1 /tmp/pmc2 > /dev/null
cat gpurun_out/probe_pmc.md
