// step_wide64.hip — the fp64 wide tier of step.hip (namespace pnp_wide64).
//
// The fp64 instantiation runs the single-env facade (pnp_amd.envs.FrankaShelfPNPEnv, the C1
// execute_pnp demo) and the batched behaviour trees (pnp_amd.batched_bt).  Its full tier holds 48
// contacts; closed fingers on a cube make more, and without a further tier the full kernel
// truncated them (MuJoCo's CONTACTFULL / CNSTRFULL).  This build holds 96 contacts, 400 rows,
// 3712 packed Jacobian slots and 4096 dense island-Jacobian entries in fp64 (~150 KB of LDS, one
// env per CU) and resumes the sub-steps the full fp64 kernel hands over (pnp_step_f64,
// pnp_env_step_f64), from the sub-step that overflowed -- the same device code and arithmetic,
// so the hand-over is exact; past these capacities it truncates with the warning bits.
#define PNP_WIDE64 1
#define PNP_NS_NAME pnp_wide64
#define PH_MAXCON 96
#define PH_MAXEFC 400
#define PH_MAXJSLOT 3712
#define PH_JTCAP 4096
#include "step.hip"

static_assert(sizeof(pnp_wide64::Env<double>) <= 163840, "fp64 wide Env must fit 1 env per CU (160 KB LDS)");
