#!/bin/bash
# fp32 precision pass: per-tree errors on identical inputs, data-vs-solver split, step parity
# tests, then the C3 step leg.  Each GPU step has its own time limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-prec}"
timeout -k 10 300 python -u tools/f32_precision.py 1 > "$OUT/${TAG}_1.log" 2>&1 || exit $?
DATA_SOLVE=1 timeout -k 10 300 python -u tools/f32_precision.py > "$OUT/${TAG}_data.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_step_gpu.py} -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" "$OUT/${TAG}_pytest.log" | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:---no-tqc --no-ik} --no-cpu-baseline > "$OUT/${TAG}_bench.log" 2>&1 || exit $?
grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_bench.log" | head -1; grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_bench.log" | head -1
