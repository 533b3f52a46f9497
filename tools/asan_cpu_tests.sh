#!/bin/bash
# Host-code sanitizer pass (CPU only): builds the oracle (oracle/*.c) and libpnp's host code
# (pnp_capi.cpp, phys_host.cpp, resident.cpp, the launchers' argument checks) with ASan + UBSan,
# then runs the CPU test suite against those builds with the clang ASan runtime preloaded.
set -u
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
LOG="${1:-$ROOT/profiles/r03/asan_cpu_tests.log}"
mkdir -p "$(dirname "$LOG")"
make -s -C oracle asan || exit $?
make -s -j8 -C mujoco-panda-pnp_amd/csrc asan > /dev/null 2>&1 || { echo "libpnp asan build failed"; exit 1; }
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# $(date -u +%FT%TZ) ASan+UBSan: oracle/liboracle_asan.so, pnp_amd/libpnp_asan.so (host code), runtime $RT"
  LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0 \
    PNP_ORACLE_LIB="$ROOT/oracle/liboracle_asan.so" PNP_LIB="$ROOT/mujoco-panda-pnp_amd/pnp_amd/libpnp_asan.so" \
    python - <<'PY'
import ctypes, os, sys
sys.path[:0] = [".", "mujoco-panda-pnp_amd"]
from pnp_amd import _lib
from oracle import oracle as O
_lib.load(); O.lib()
maps = open("/proc/self/maps").read()
for so in ("libpnp_asan.so", "liboracle_asan.so", "libclang_rt.asan"):
    print(f"loaded {so}: {so in maps}")
PY
  LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    PNP_ORACLE_LIB="$ROOT/oracle/liboracle_asan.so" PNP_LIB="$ROOT/mujoco-panda-pnp_amd/pnp_amd/libpnp_asan.so" \
    timeout -k 10 1800 python -m pytest tests -q -m "not gpu" -p no:cacheprovider 2>&1
  echo "exit: $?"
} > "$LOG"
tail -3 "$LOG"
# the sanitizer builds are CPU-only artefacts: not left in the tree that travels to the GPU box
rm -f "$ROOT/oracle/liboracle_asan.so" "$ROOT/mujoco-panda-pnp_amd/pnp_amd/libpnp_asan.so"
