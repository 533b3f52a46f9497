#!/bin/bash
# One launcher for every GPU-box pass (run through gpurun: `gpurun -- 'TAG=x bash tools/gpu.sh
# <step> ...'`).  Each GPU step runs under its own time limit and writes gpurun_out/${TAG}_<name>.log;
# a fault, abort, timeout or (except pytest's "tests failed" = 1) any non-zero exit ends the script.
# Steps, run in the order given (several per call):
#   tests [pytest args]   every -m gpu test (or the given node ids / -k), per-tree bars printed
#   smoke                 __graft_entry__.smoke()
#   bench [bench args]    the default bench (CPU baseline included unless --no-cpu-baseline)
#   trace                 rocprofv3 kernel trace + stats of the bench's step and gym legs
#   steadytrace           the same for the gym leg's steady state (50 burn-in steps, 5 timed)
#   pmc                   PMC HBM traffic of the step kernel (FETCH_SIZE, WRITE_SIZE: separate passes)
#   sq                    SQ counters of the step kernel (two passes of 8) + tools/sq_summary.py
#   stage                 per-stage shader-clock profile on the bench's inputs (tools/step_parity.py)
#   tqcprof               rocprofv3 kernel trace of the fused TQC learner step
#   tool <script> [args]  a python diagnostic (tools/*.py) -- all remaining arguments are its own
#   ab                    library A/B: state digests of the tree's libpnp.so and of each $ALTS .so
#                         (PNP_LIB; an <alt>.so.env file beside it is sourced for that alternative's
#                         runs), then the C3 and gym legs interleaved twice
#   evidence              tests smoke bench trace pmc sq stage tqcprof
# (Round 5's 43 one-off gpu_*.sh launchers were folded into this script; older profiles name them,
# their text is in the git history.)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-g}"
export TMPDIR=/tmp
BENCH_STEP="--steps 5 --warmup 1 --no-cpu-baseline --no-gym --no-ik --no-tqc"

run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && ! { [ "$name" = tests ] && [ $rc -eq 1 ]; }; then exit $rc; fi
}
prof() {  # rocprofv3 from /tmp with the program itself after -- (no launcher hops)
  local name=$1 t=$2; shift 2
  (cd /tmp && timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/${TAG}_$name.log" 2>&1)
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/${TAG}_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}

do_step() {
  local s=$1; shift
  case "$s" in
    tests)
      if [ $# -gt 0 ]; then run tests 1100 python -u -m pytest "$@" -m gpu -v -s --timeout 240 --timeout-method thread
      else run tests 1100 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread; fi
      grep -E "FAILED|worst error" "$OUT/${TAG}_tests.log" | cut -c1-300 | head -40 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 700 python -u bench.py "$@"; tail -1 "$OUT/${TAG}_bench.log" | cut -c1-600 ;;
    trace)
      prof trace 600 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- \
        python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-tqc --no-ik --steady-burn 0 ;;
    steadytrace)
      prof steadytrace 600 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_sprof" -o run -- \
        python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-tqc --no-ik --steady-burn 50 ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        prof pmc_$c 300 --pmc $c --output-format csv -d "$OUT/${TAG}_pmc_$c" -o run -- python3 "$ROOT/bench.py" $BENCH_STEP
      done
      python3 tools/pmc_traffic.py "$OUT/${TAG}_pmc_FETCH_SIZE" "$OUT/${TAG}_pmc_WRITE_SIZE" "pnp_compact::step_kernel" 4096 \
        "$OUT/${TAG}_pmc_traffic.json" 5 > "$OUT/${TAG}_pmc_traffic.log" 2>&1; tail -3 "$OUT/${TAG}_pmc_traffic.log" ;;
    sq)
      local P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
      local P2="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
      prof sq_p1 180 --pmc $P1 --output-format csv -d "$OUT/${TAG}_sq_p1" -o run -- python3 "$ROOT/bench.py" $BENCH_STEP
      prof sq_p2 180 --pmc $P2 --output-format csv -d "$OUT/${TAG}_sq_p2" -o run -- python3 "$ROOT/bench.py" $BENCH_STEP
      python3 tools/sq_summary.py "$OUT/${TAG}_sq_p1" "$OUT/${TAG}_sq_p2" "pnp_compact::step_kernel<float, false>" \
        --json "$OUT/${TAG}_sq.json" --waves-per-simd 2 > "$OUT/${TAG}_sq_summary.txt" 2>&1; tail -12 "$OUT/${TAG}_sq_summary.txt" ;;
    stage) run stage 300 python3 -u tools/step_parity.py 4096 prof bench ;;
    tqcprof)
      prof tqcprof 300 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_tqc_prof" -o run -- \
        python3 "$ROOT/tools/tqc_learner_bench.py" fused 200 ;;
    ab)
      run digest_tree 300 python3 -u tools/state_digest.py 512
      for a in ${ALTS:-}; do
        local n; n=$(basename "$a" .so)
        ( if [ -f "$ROOT/$a.env" ]; then . "$ROOT/$a.env"; fi
          PNP_LIB="$ROOT/$a" run digest_$n 300 python3 -u tools/state_digest.py 512 ) || exit $?
        if diff <(grep -v amdgpu "$OUT/${TAG}_digest_tree.log") <(grep -v amdgpu "$OUT/${TAG}_digest_$n.log") > /dev/null
        then echo "$n: digests identical"; else echo "$n: DIGESTS DIFFER"; fi
      done
      for i in 1 2; do
        for a in tree ${ALTS:-}; do
          local n; n=$(basename "$a" .so)
          if [ "$a" = tree ]; then unset PNP_LIB; else export PNP_LIB="$ROOT/$a"; fi
          # an alternative's own environment (runtime switches), from <alt>.env next to it
          unset PNP_GYM_FULL_MW PNP_GYM_WIDE_PCT PNP_GYM_FULL_PCT PNP_GYM_ROUTE_ORDER PNP_GYM_WIDE_GRID
          if [ "$a" != tree ] && [ -f "$ROOT/$a.env" ]; then . "$ROOT/$a.env"; fi
          run ab_${n}_$i 400 python -u bench.py --steps 20 --warmup 3 --no-tqc --no-ik --no-cpu-baseline ${AB_ARGS:-}
          echo "$n run $i: $(tail -1 "$OUT/${TAG}_ab_${n}_$i.log" | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["value"]/1e6,3), "M C3;", round(r["gym"]["gym_steps_per_s"]), "gym", ((r["gym"].get("steady") or {}).get("ms_per_gym_step")), "ms steady")' 2>/dev/null)"
        done
      done
      unset PNP_LIB ;;
    evidence)
      for x in tests smoke bench trace pmc sq stage tqcprof; do do_step $x; done ;;
    *) echo "tools/gpu.sh: unknown step '$s'"; exit 2 ;;
  esac
}

if [ $# -eq 0 ]; then set -- evidence; fi
case "$1" in
  tool) shift; n=$(basename "$1" .py); run "tool_$n" "${TOOL_TIMEOUT:-300}" python3 -u "$@"; exit 0 ;;
  tests|bench) s=$1; shift; do_step "$s" "$@"; exit 0 ;;
esac
for s in "$@"; do do_step "$s"; done
echo "all done"
