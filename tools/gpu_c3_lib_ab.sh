#!/bin/bash
# C3 library A/B: the state digests of the in-tree libpnp.so and of each library in $ALTS (PNP_LIB)
# must match; then the bench's C3 leg, interleaved twice
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-c3lab}"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/state_digest.py 512 > "$OUT/${TAG}_digest_tree.log" 2>&1 || { tail -5 "$OUT/${TAG}_digest_tree.log"; exit 1; }
for a in $ALTS; do
  n=$(basename $a .so)
  PNP_LIB="$ROOT/$a" timeout -k 10 300 python3 -u tools/state_digest.py 512 > "$OUT/${TAG}_digest_$n.log" 2>&1 || { tail -5 "$OUT/${TAG}_digest_$n.log"; exit 1; }
  if diff <(grep -v amdgpu "$OUT/${TAG}_digest_tree.log") <(grep -v amdgpu "$OUT/${TAG}_digest_$n.log") > /dev/null; then echo "$n: digests identical"; else echo "$n: DIGESTS DIFFER"; fi
done
for i in 1 2; do
  for a in tree $ALTS; do
    n=$(basename $a .so)
    if [ $a = tree ]; then unset PNP_LIB; else export PNP_LIB="$ROOT/$a"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-gym --no-tqc --no-ik --no-cpu-baseline > "$OUT/${TAG}_${n}_$i.log" 2>&1 || { tail -5 "$OUT/${TAG}_${n}_$i.log"; exit 1; }
    echo "$n run $i: $(grep -o '"value": [0-9.e+]*' "$OUT/${TAG}_${n}_$i.log" | head -1)"
  done
done
unset PNP_LIB
