#!/bin/bash
# PMC HBM traffic of the bench's step kernel (FETCH_SIZE and WRITE_SIZE in separate passes) and
# the per-stage shader-clock profile.  Each GPU step has its own time limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${TAG:-pmc}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/${TAG}_$c" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc > "$OUT/${TAG}_$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT/${TAG}_FETCH_SIZE" "$OUT/${TAG}_WRITE_SIZE" "pnp_compact::step_kernel" 4096 "$OUT/${TAG}_traffic.json" 5
timeout -k 10 300 python3 -u tools/step_parity.py 4096 prof > "$OUT/${TAG}_stageprof.log" 2>&1
rc=$?; head -40 "$OUT/${TAG}_stageprof.log"; exit $rc
