set -u
VARIANTS=noeul TAG=lab4 bash tools/gpu_lib_ab.sh || exit $?
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/gym_profile.py 4096 4 uniform > gpurun_out/gp5_uniform.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/gym_profile.py 4096 4 saturated > gpurun_out/gp5_sat.log 2>&1 || exit $?
tail -12 gpurun_out/gp5_sat.log
