// step_compact.hip — the compact-capacity build of step.hip's fp32 step kernel.
//
// Same device code as step.hip (namespace pnp_compact), with capacities sized for the scene's
// common case instead of its worst case: 20 contacts (settled scene: 12), 256 broadphase
// survivors, 96 constraint rows, 800 packed Jacobian slots, 768 dense island-Jacobian entries and
// 288 packed island-Hessian entries.  The per-env LDS working set (Env, laid out by lifetime) is
// then 20.1 KB: 8 envs per CU, two waves on every SIMD, so 4096 envs run in 2 rounds of 2048
// resident waves (the full build: 3 envs per CU).  Registers are budgeted for two waves per SIMD
// (<= 256 VGPR + AGPR).  An env whose sub-step would overflow one of these capacities stops before
// that sub-step changes its state and is finished by the full kernel's resume pass (step.hip:
// launch_step, PNP_RESUME_*), so results are the full kernel's.
#define PNP_COMPACT 1
#define PH_MAXCON 20
#define PH_MAXEFC 96
#define PH_MAXJSLOT 800
#define PH_HCAP 288
#define PH_MAXLIVE 256
#define PH_JTCAP 768
#define PNP_STEP_WAVES 2
#include "step.hip"

static_assert(sizeof(pnp_compact::Env<float>) <= 20480, "compact Env must fit 8 envs per CU (160 KB LDS)");
