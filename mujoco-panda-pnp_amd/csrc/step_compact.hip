// step_compact.hip — the compact-capacity build of step.hip's fp32 step kernel.
//
// Same device code as step.hip (namespace pnp_compact), with capacities sized for the scene's
// common case instead of its worst case: 20 contacts (settled scene: 12), 96 constraint rows,
// 1000 packed Jacobian slots, 768 dense island-Jacobian entries.  The per-env LDS working set is
// then 26.3 KB instead of 38.7 KB: 6 envs per CU instead of 4, two waves on half of the SIMDs,
// so 4096 envs run in 3 rounds of resident waves instead of 4.  Registers are budgeted for two
// waves per SIMD (<= 256 VGPR + AGPR).  An env whose sub-step would overflow one of these
// capacities stops before that sub-step changes its state and is finished by the full kernel's
// resume pass (step.hip: launch_step, PNP_RESUME_*), so results are the full kernel's.
#define PNP_COMPACT 1
#define PH_MAXCON 20
#define PH_MAXEFC 96
#define PH_MAXJSLOT 1000
#define PH_JTCAP 768
#define PNP_STEP_WAVES 2
#include "step.hip"

static_assert(sizeof(pnp_compact::Env<float>) <= 26624, "compact Env must fit 6 envs per CU (160 KB LDS)");
