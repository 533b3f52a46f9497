#!/bin/bash
# gym tier-capacity check: the env GPU tests, the bench's gym leg twice, the per-step queue census.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-cap}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_bench_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_bench_$i.log"; exit 1; }
  echo "run $i: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_bench_$i.log" | head -1) $(grep -o '"ms_per_gym_step": [0-9.e+]*' "$OUT/${TAG}_bench_$i.log" | head -1)"
done
timeout -k 10 300 python -u tools/gym_queue_census.py 4096 ${NSTEP:-6} > "$OUT/${TAG}_census.log" 2>&1 || { tail -5 "$OUT/${TAG}_census.log"; exit 1; }
grep -v amdgpu "$OUT/${TAG}_census.log" | cut -c1-230
