#!/bin/bash
# Write-back check on the current tree (item 7): the C3 step tests, the step leg of the bench,
# PMC WRITE_SIZE / FETCH_SIZE (separate passes) and SQ pass 1 of the compact step kernel.  Each GPU
# step under its own time limit; the first failure ends the script.
set -eu
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-wb}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
tail -1 "$OUT/${TAG}_pytest.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-gym --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1
grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_bench.log" | head -1
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d "$OUT/${TAG}_pmc_$c" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc > "$OUT/${TAG}_pmc_$c.log" 2>&1
done
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  --output-format csv -d "$OUT/${TAG}_sq_p1" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc > "$OUT/${TAG}_sq_p1.log" 2>&1
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT/${TAG}_pmc_FETCH_SIZE" "$OUT/${TAG}_pmc_WRITE_SIZE" "pnp_compact::step_kernel" 4096 \
  "$OUT/${TAG}_pmc_traffic.json" 5 2>&1 | tail -2
python3 tools/sq_summary.py "$OUT/${TAG}_sq_p1" "$OUT/${TAG}_sq_p1" "pnp_compact::step_kernel<float, false>" --waves-per-simd 2 2>&1 | grep -E "WAIT_ANY /|VALU pipe" || true
