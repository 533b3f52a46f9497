// env_compact.hip — the compact-capacity tier of the fp32 gym step (FrankaEnv.step fused).
//
// step.hip's device code at step_compact.hip's capacities (20 contacts, 96 rows, 800 slots: 8 envs
// per CU) with the gym kernels of env_dev.h, in a namespace and constant image of its own.  A
// translation unit of its own too: compiled into step_compact.hip, the gym kernels grew the
// compact step kernel's call frames (384 -> 464 B per lane) and its write-back traffic 5x.  The
// full build's launch_env_step runs this kernel over every env, then the full and the wide
// tiers' resume passes over the envs handed over (step.hip: PNP_RESUME_*).
#define PNP_COMPACT 1
#define PNP_GYM 1
#define PNP_NS_NAME pnp_compact_gym
#define PH_MAXCON 20
#define PH_MAXEFC 96
#define PH_MAXJSLOT 800
#define PH_HCAP 288
#define PH_MAXLIVE 256
#define PH_JTCAP 768
#define PNP_STEP_WAVES 2
#include "step.hip"

static_assert(sizeof(pnp_compact_gym::Env<float>) <= 20480, "compact gym Env must fit 8 envs per CU (160 KB LDS)");
static_assert(PH_MAXCON == PNP_GC_MAXCON && PH_MAXEFC == PNP_GC_MAXEFC && PH_MAXJSLOT == PNP_GC_MAXJSLOT &&
                  PH_JTCAP == PNP_GC_JTCAP && PH_HCAP == PNP_GC_HCAP,
              "env_dev.h's routing estimate (tier_need) must see this tier's capacities");
