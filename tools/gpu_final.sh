#!/bin/bash
# Round evidence on the final tree, one GPU-box pass: GPU tests, smoke, the default bench (CPU
# baseline included), a rocprofv3 kernel trace of the bench, PMC traffic (FETCH_SIZE / WRITE_SIZE
# in separate passes) + stage cycles, and the gym-step resume-pass A/B.  Every GPU step has its
# own time limit; a fault, abort or timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-final}"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/${TAG}_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cd /tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-tqc
cd "$ROOT"
TAG=${TAG}_pmc bash tools/gpu_pmc.sh > "$OUT/${TAG}_pmc.log" 2>&1 || { echo "pmc rc=$?"; exit 1; }
tail -3 "$OUT/${TAG}_pmc.log"
for v in 1 0 1 0; do
  step fr$v 300 env PNP_GYM_FULL_RESUME=$v python bench.py --steps 5 --warmup 2 --no-tqc --no-ik --no-cpu-baseline
done
echo "all done"
