#!/bin/bash
# Heavy-env check: step / env GPU tests (tier and routing exactness), the bench's step and gym
# legs, and the gym stage profile under saturated actions (tools/gym_profile.py).  Each GPU step
# has its own time limit; the script stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-heavy}"
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_step_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
echo "$(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_bench.log")  C3 $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_bench.log" | head -1)"
timeout -k 10 240 python -u tools/gym_profile.py 4096 4 saturated > "$OUT/${TAG}_gp_sat.log" 2>&1 || exit $?
grep -E "envs with|noslip_W" "$OUT/${TAG}_gp_sat.log" | tail -4
