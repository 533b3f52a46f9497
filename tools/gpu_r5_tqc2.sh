#!/bin/bash
# round 5: fused learner tests + timing + SQ counters of its kernels; the full tier's stage profile
# on the gym's closed-gripper states.  Each GPU step under its own limit; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TAG="${TAG:-r5t2}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tqc_gpu.py -k fused > "$OUT/${TAG}_tests.log" 2>&1 || { tail -20 "$OUT/${TAG}_tests.log"; exit 1; }
tail -1 "$OUT/${TAG}_tests.log"
timeout -k 10 120 python3 tools/tqc_learner_bench.py fused 300 > "$OUT/${TAG}_bench.log" 2>&1 || exit 1
grep fused "$OUT/${TAG}_bench.log" | cut -c1-60
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
P3="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_MFMA_F32 SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_VMEM SQ_ACTIVE_INST_FLAT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/${TAG}_sq$i" -o run -- python3 "$ROOT/tools/tqc_learner_bench.py" fused 30 > "$OUT/${TAG}_sq$i.log" 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/${TAG}_sq$i.log"; }
done
cd "$ROOT"
for k in tqc_fwd_kernel tqc_pi_critic_kernel tqc_wgrad_adam_kernel; do
  python3 tools/sq_summary.py "$OUT/${TAG}_sq1" "$OUT/${TAG}_sq2" "$OUT/${TAG}_sq3" $k --waves-per-simd 2 > "$OUT/${TAG}_sq_$k.txt" 2>&1
  grep -E "per wave|VALU_MFMA|INSTS_VALU |INSTS_LDS |WAIT_ANY /|ACTIVE_INST_ANY /|BANK|VMEM_RD |WAIT_INST_VMEM|SALU " "$OUT/${TAG}_sq_$k.txt" | head -14
done
timeout -k 10 200 python3 -u tools/full_tier_profile.py scratch/handover_states_s4.npz 1024 10 > "$OUT/${TAG}_fullprof.log" 2>&1 || { tail -5 "$OUT/${TAG}_fullprof.log"; exit 1; }
grep -v amdgpu.ids "$OUT/${TAG}_fullprof.log" | head -40
