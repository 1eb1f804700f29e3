set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_ramp -o run -- python3 bench.py --steps 150 --warmup 0 > gpurun_out/ramp_prof.log 2>&1
db=$(find /tmp/prof_ramp -name '*.db' | head -1)
python tools/prof_ramp.py "$db" lstm_small_bwd_gs_kernel > gpurun_out/ramp_bwd.txt
python tools/prof_ramp.py "$db" lstm_small_fwd_gs_kernel > gpurun_out/ramp_fwd.txt
paste gpurun_out/ramp_fwd.txt gpurun_out/ramp_bwd.txt | head -40
