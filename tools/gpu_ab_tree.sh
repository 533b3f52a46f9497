#!/bin/bash
# A/B against another source tree shipped under ab/<name> (built on the CPU beforehand): the C3
# step leg (bench.py --no-gym --no-tqc --no-ik) and the stage-cycle profile, current tree first,
# then each tree in $TREES, twice, interleaved.  GYM=1 keeps the bench's gym leg (its
# gym-steps/s printed too).  Each GPU step has its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-abt}"
GYMARG=--no-gym; [ -z "${GYM:-}" ] || GYMARG=
export TMPDIR=/tmp
for i in 1 2; do
  for t in cur ${TREES:-v19}; do
    d="$ROOT"; [ "$t" = cur ] || d="$ROOT/ab/$t"
    (cd "$d" && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 $GYMARG --no-tqc --no-ik --no-cpu-baseline ${BENCHARGS:-}) > "$OUT/${TAG}_${t}_bench$i.log" 2>&1 || exit $?
    echo "$t run $i: $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${t}_bench$i.log" | head -1) $(grep -o '"gym_steps_per_s": [0-9.e+]*' "$OUT/${TAG}_${t}_bench$i.log" | head -1)"
    if [ $i -eq 1 ]; then
      (cd "$d" && timeout -k 10 300 python3 -u tools/step_parity.py 4096 prof) > "$OUT/${TAG}_${t}_stageprof.log" 2>&1 || exit $?
      grep -m1 "cycles" "$OUT/${TAG}_${t}_stageprof.log"
    fi
  done
done
