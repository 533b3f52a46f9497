#!/bin/bash
# adaptive wide-consumer count (PNP_GYM_QUEUE_PCT): env GPU tests, then per value in $PCTS the bench's gym
# leg and the per-step queue census over $NSTEP steps
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-qp}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for pct in ${PCTS:-100 200}; do
  PNP_GYM_QUEUE_PCT=$pct timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_$pct.log" 2>&1 || { tail -5 "$OUT/${TAG}_$pct.log"; exit 1; }
  echo "pct $pct: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_$pct.log" | head -1)"
  PNP_GYM_QUEUE_PCT=$pct timeout -k 10 300 python -u tools/gym_queue_census.py 4096 ${NSTEP:-10} > "$OUT/${TAG}_census_$pct.log" 2>&1 || { tail -5 "$OUT/${TAG}_census_$pct.log"; exit 1; }
  grep -v amdgpu "$OUT/${TAG}_census_$pct.log" | sed 's/started.*queue {.published.: \([0-9]*\).*next/pub \1 next/' | cut -c1-50 | tr '\n' ';'; echo
done
