// step_wide.hip — the wide-capacity build of step.hip's fp32 kernels (namespace pnp_wide).
//
// Same device code as step.hip with capacities for the contact-rich states of the gym workload:
// closed fingers pressed together (or onto a shelf board) make 50-150 contacts — box-box pad
// pairs with up to 8 points each, finger-mesh / pad / board pairs with up to 5 each (multiccd) —
// where the full build stops at 48.  192 contacts (the CPU oracle's capacity, oracle/physics.h;
// tools/contact_census.py: up to 143 in 64 envs x 6 saturated-action gym steps), 784 constraint
// rows (6 weld + 9 joint limits + 4 x 192 pyramid edges), 7168 packed Jacobian slots and 8192
// dense island-Jacobian entries (an arm + cube island of 15 dofs with ~500 rows keeps the dense
// path): ~133 KB of LDS per env, 1 env per CU.  It only runs the envs the full kernel hands over
// (pnp_step's and pnp_env_step's resume passes: step.hip launch_step, env_dev.h launch_env_step),
// from the sub-step that overflowed; past these capacities it truncates like MuJoCo with a full
// buffer (warning bits CONTACTFULL / CNSTRFULL).
#define PNP_WIDE 1
#define PH_MAXCON 192
#define PH_MAXEFC 784
#define PH_MAXJSLOT 7168
#define PH_JTCAP 8192
#include "step.hip"

static_assert(sizeof(pnp_wide::Env<float>) <= 163840, "wide Env must fit 1 env per CU (160 KB LDS)");
