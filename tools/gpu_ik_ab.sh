set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ik_gpu.py tests/test_skills_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ik_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ik_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/ik_pytest.log | head -20; exit $rc; }
timeout -k 10 200 python -u bench.py --workload ik --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ik_bench_group.log 2>&1 || exit $?
PNP_IK_SERIAL=1 timeout -k 10 200 python -u bench.py --workload ik --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ik_bench_serial.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --workload ik --regime ik_test --params ik_test --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ik_bench_group_iktest.log 2>&1 || exit $?
PNP_IK_SERIAL=1 timeout -k 10 200 python -u bench.py --workload ik --regime ik_test --params ik_test --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ik_bench_serial_iktest.log 2>&1 || exit $?
for f in gpurun_out/ik_bench_*.log; do echo $f; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ik_stats'])"; done
