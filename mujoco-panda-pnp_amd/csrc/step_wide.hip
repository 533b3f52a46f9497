// step_wide.hip — the wide-capacity build of step.hip's fp32 kernels (namespace pnp_wide).
//
// Same device code as step.hip with capacities for the contact-rich states of the gym workload:
// closed fingers pressed together (or onto a shelf board) make 50-100 contacts — box-box pad
// pairs with up to 8 points each, finger-mesh / pad pairs — where the full build stops at 48.
// 96 contacts (the CPU oracle's capacity, oracle/physics.h), 400 constraint rows (6 weld + 9
// joint limits + 4 x 96 pyramid edges), 4096 packed Jacobian slots and 5120 dense island-Jacobian
// entries (an arm + cube island of 15 dofs with ~300 rows keeps the dense path): ~77 KB of LDS per
// env, 2 envs per CU.  It only runs the envs the full kernel hands over
// (pnp_step's and pnp_env_step's resume passes: step.hip launch_step, env_dev.h launch_env_step),
// from the sub-step that overflowed; past these capacities it truncates like MuJoCo with a full
// buffer (warning bits CONTACTFULL / CNSTRFULL).
#define PNP_WIDE 1
#define PH_MAXCON 96
#define PH_MAXEFC 400
#define PH_MAXJSLOT 4096
#define PH_JTCAP 5120
#include "step.hip"

static_assert(sizeof(pnp_wide::Env<float>) <= 81920, "wide Env must fit 2 envs per CU (160 KB LDS)");
