#!/bin/bash
# Hand-over queue check (gym step): env GPU tests, then the gym leg of the bench with the queue
# off / on at consumer grids $GRIDS, twice each.  Each GPU step has its own time limit; the first
# failure ends the script.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-hq}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
tail -1 "$OUT/${TAG}_pytest.log"
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_$lab.log" 2>&1
  echo "$lab: $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_$lab.log" | head -1) $(grep -o '"max_warn": [0-9]*' "$OUT/${TAG}_$lab.log" | head -1)"
}
for i in 1 2; do
  run off$i PNP_GYM_QUEUE=0
  for g in ${GRIDS:-64}; do run q${g}_$i PNP_GYM_QUEUE_CU=$g; done
done
