set -e
bash tools/gpu_sw_pmc.sh mbpmc7 1440 7
bash tools/gpu_sw_pmc.sh mbpmc3 1440 3
