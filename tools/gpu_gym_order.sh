#!/bin/bash
# full resume pass ordering A/B (PNP_GYM_FULL_ORDER): env GPU tests, then the bench's gym leg with
# the order on / off, interleaved twice
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-ord}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
for i in 1 2; do
  for o in 1 0; do
    PNP_GYM_FULL_ORDER=$o timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${o}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${o}_$i.log"; exit 1; }
    echo "order $o run $i: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${o}_$i.log" | head -1)"
  done
done
