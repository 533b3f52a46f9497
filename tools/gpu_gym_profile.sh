set -u
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/gym_profile.py 4096 4 uniform > gpurun_out/gp_uniform.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/gym_profile.py 4096 4 saturated > gpurun_out/gp_sat.log 2>&1 || exit $?
PNP_STEP_COMPACT=0 timeout -k 10 240 python -u tools/gym_profile.py 4096 4 uniform > gpurun_out/gp_uniform_full.log 2>&1 || exit $?
