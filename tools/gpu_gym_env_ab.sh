#!/bin/bash
# Gym-step env-switch A/B on one library: tests with VAR=B (the candidate), then the bench gym
# leg interleaved twice for VAR=A and VAR=B, and a kernel trace of the gym leg under VAR=B.
# usage: VAR=PNP_GYM_FULL_RESUME A=1 B=0 TESTS="tests/test_env_gpu.py" bash tools/gpu_gym_env_ab.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-geab}"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  env "$VAR=$B" timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
fi
for rep in 1 2; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_bench$rep.log" 2>&1 || exit $?
    echo "$VAR=$v run $rep: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_bench$rep.log" | head -1)"
  done
done
cd /tmp
export "$VAR=$B"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_trace.log" 2>&1 || exit $?
cd "$ROOT"
python3 tools/gym_trace_summary.py "$(find "$OUT/${TAG}_trace" -name '*kernel_trace.csv' | head -1)" 12
