#!/bin/bash
# SQ counters of the bench's step leg (stall split and instruction mix), two passes of 8 SQ
# counters each, one rocprofv3 run per pass; then tools/sq_summary.py.  Stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${TAG:-sq}"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/${TAG}_counters.txt" 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d "$OUT/${TAG}_p$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc > "$OUT/${TAG}_p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/${TAG}_p$i.log"; exit $rc; }
done
cd "$ROOT"
python3 tools/sq_summary.py "$OUT/${TAG}_p1" "$OUT/${TAG}_p2" "pnp_compact::step_kernel<float, false>" --json "$OUT/${TAG}_sq.json" --waves-per-simd 2 > "$OUT/${TAG}_summary.txt"
cat "$OUT/${TAG}_summary.txt"
