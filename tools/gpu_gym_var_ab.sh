#!/bin/bash
# env-variable A/B of the bench's gym leg: the env GPU tests, then $VAR at each value in $VALS,
# interleaved twice; then (NSTEP > 0) the per-step queue census per value
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-vab}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -1 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for i in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${v}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${v}_$i.log"; exit 1; }
    echo "$VAR=$v run $i: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${v}_$i.log" | head -1)"
  done
done
if [ "${NSTEP:-0}" -gt 0 ]; then
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python -u tools/gym_queue_census.py 4096 $NSTEP > "$OUT/${TAG}_census_$v.log" 2>&1 || { tail -5 "$OUT/${TAG}_census_$v.log"; exit 1; }
    echo "$VAR=$v:"; grep -v amdgpu "$OUT/${TAG}_census_$v.log" | sed 's/np.int64(\([0-9]*\))/\1/g; s/queue {.published.: \([0-9]*\).*next/pub \1 next/' | cut -c1-120
  done
fi
