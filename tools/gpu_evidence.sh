#!/bin/bash
# Round evidence on the current tree, one GPU-box pass (each GPU step under its own time limit; a
# fault, abort or timeout ends the script):
#   1. every GPU test, 2. smoke(), 3. the default bench (CPU baseline included),
#   4. rocprofv3 kernel trace + stats of the bench's step and gym legs,
#   5. PMC HBM traffic of the step leg (FETCH_SIZE and WRITE_SIZE in separate passes),
#   6. SQ counters of the step leg (two passes of 8), 7. the stage-cycle profile on bench inputs,
#   8. rocprofv3 kernel trace of the fused TQC learner step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-ev}"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...  (pytest's exit 1 = test failures: reported, the script goes on)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/${TAG}_$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && ! { [ "$name" = pytest ] && [ $rc -eq 1 ]; }; then exit $rc; fi
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest 1100 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python -u bench.py
cd /tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-tqc --no-ik
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/${TAG}_pmc_$c" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc
done
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  step sq_p$i 180 rocprofv3 --pmc $P --output-format csv -d "$OUT/${TAG}_sq_p$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc
done
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT/${TAG}_pmc_FETCH_SIZE" "$OUT/${TAG}_pmc_WRITE_SIZE" "pnp_compact::step_kernel" 4096 \
  "$OUT/${TAG}_pmc_traffic.json" 5 > "$OUT/${TAG}_pmc_traffic.log" 2>&1; tail -3 "$OUT/${TAG}_pmc_traffic.log"
python3 tools/sq_summary.py "$OUT/${TAG}_sq_p1" "$OUT/${TAG}_sq_p2" "pnp_compact::step_kernel<float, false>" \
  --json "$OUT/${TAG}_sq.json" --waves-per-simd 2 > "$OUT/${TAG}_sq_summary.txt" 2>&1; tail -12 "$OUT/${TAG}_sq_summary.txt"
step stageprof 300 python3 -u tools/step_parity.py 4096 prof bench
cd /tmp
# the fused TQC learner step (C5 at train.py's update ratio is ~all learner): kernel trace
step tqc_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_tqc_prof" -o run -- \
  python3 "$ROOT/tools/tqc_learner_bench.py" fused 200
cd "$ROOT"
echo "all done"
