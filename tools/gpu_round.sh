#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a step that faults/aborts/times out (rc not in {0,1}) ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    tqc)   run pytest_tqc 300 python -u -m pytest tests/test_tqc_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    prof)  cd /tmp && run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-tqc; cd "$ROOT" ;;
    pmc)   cd /tmp && run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-tqc && \
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-tqc; cd "$ROOT" ;;
  esac
done
echo "all steps done"
