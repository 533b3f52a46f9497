#!/bin/bash
# Gym-step tiers A/B: env GPU tests, then the gym profile starting in the compact tier vs the full tier.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-gab}"
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_tqc_gpu.py tests/test_skills_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for mode in 1 0; do
  for act in uniform saturated; do
    PNP_GYM_COMPACT=$mode timeout -k 10 300 python -u tools/gym_profile.py 4096 4 $act > "$OUT/${TAG}_gym_${act}_c$mode.log" 2>&1 || exit $?
    echo "compact=$mode $act"; head -6 "$OUT/${TAG}_gym_${act}_c$mode.log" | grep "gym step\|CONTACTFULL"
  done
done
