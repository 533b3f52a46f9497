// LDS budget of the per-env working set (step.hip Env<float>), per capacity build: every field with
// its bytes, offset and the stages between which it is live.  Host-only
// program (offsetof / sizeof of the device struct); build one capacity at a time like the kernels:
//   hipcc -std=c++17 --offload-arch=gfx950 -DPNP_COMPACT=1 -DPH_MAXCON=20 -DPH_MAXEFC=96 \
//     -DPH_MAXJSLOT=800 -DPH_HCAP=288 -DPH_MAXLIVE=256 -DPH_JTCAP=768 -DPNP_STEP_WAVES=2 \
//     -I mujoco-panda-pnp_amd/csrc tools/env_lds_table.hip -o /tmp/env_lds && /tmp/env_lds
// (tools/env_lds_table.sh builds and runs it for the compact, full and wide builds.)
#include <cstddef>
#include <cstdio>
#include "step.hip"

#define F(f, live) row(#f, offsetof(E, f), sizeof(((E*)0)->f), live)
using E = PNP_NS::Env<float>;
static size_t tot = 0;
static void row(const char* n, size_t off, size_t sz, const char* live) {
  printf("| %-28s | %6zu | %6zu | %s |\n", n, sz, off, live);
  tot += sz;
}
int main() {
  printf("sizeof(Env<float>) = %zu B (LDS per env); envs per CU at 160 KB: %zu\n\n", sizeof(E), (size_t)163840 / sizeof(E));
  printf("| field | bytes | offset | live (stages) |\n|---|---|---|---|\n");
  F(c_tree_dofadr, "launch (model tables)"); F(c_tree_dofnum, "launch"); F(c_tree_moff, "launch"); F(c_dof_tree, "launch");
  F(qpos, "state"); F(qvel, "state"); F(ctrl, "state"); F(mocap_pos, "state"); F(mocap_quat, "state"); F(qacc_ws, "state");
  F(wpose, "kinematics -> constraints (weld residual in fp64)");
  F(xpos, "union pos: kinematics -> velocity / gym epilogue"); F(xquat, "union pos"); F(xmat, "union pos");
  F(subcom, "union pos"); F(cdof, "union pos"); F(cinert, "union pos");
  F(gpos, "union pos.geom: kinematics -> collision"); F(gmat, "union pos.geom");
  F(xipos, "union pos.geom.crb: kinematics -> CRB"); F(xanchor, "union pos.geom.crb"); F(xaxis, "union pos.geom.crb");
  F(crb, "union pos.geom.crb"); F(scr6a, "union pos.geom.crb");
  F(con, "union pos.geom (over crb): collision -> constraint rows");
  F(cvel, "union pos.vel (over geom): velocity -> actuation"); F(cdofdot, "union pos.vel"); F(scr6, "union pos.vel");
  F(scr6b, "union pos.vel");
  F(jt, "union sol (over pos): island build -> Newton / noslip / finish");
  F(Hp, "union sol.newton"); F(ntmp, "union sol.newton"); F(rr_f, "union sol.newton"); F(rr_d, "union sol.newton");
  F(NL, "union sol.newton");
  F(efc_Wv, "union sol.noslip (over newton)"); F(ns_list, "union sol.noslip"); F(ns_len, "union sol.noslip"); F(rr_g, "union sol.noslip");
  F(M, "CRB -> Euler"); F(L, "factor M -> Euler");
  F(qfrc_smooth, "actuation -> finish"); F(qacc_smooth, "actuation -> noslip"); F(qacc, "Newton -> Euler"); F(x, "Newton");
  F(grad, "Newton"); F(p, "Newton"); F(v1, "Newton / noslip / Euler scratch"); F(v2, "noslip / finish scratch");
  F(efc_t0, "constraints -> finish"); F(efc_t1, "constraints -> finish"); F(efc_type, "constraints -> finish");
  F(efc_id, "constraints -> finish"); F(efc_act, "Newton"); F(efc_off, "constraints -> finish");
  F(efc_Jv, "constraints -> finish (union: collision staging)"); F(cst_val, "union efc_Jv: collision staging");
  F(cst_key, "union efc_Jv"); F(live, "union efc_Jv: broadphase survivors");
  F(efc_D, "constraints -> Newton"); F(efc_aref, "constraints -> Newton (fp32 noslip: Newton forces)");
  F(efc_bb, "velocity -> noslip"); F(efc_force, "Newton -> finish"); F(efc_jar, "Newton (noslip tables)");
  F(efc_Jp, "constraints -> Newton (noslip tables)");
  F(con_rbase, "constraints -> noslip"); F(con_sbase, "constraints"); F(con_t, "constraints"); F(con_dim, "constraints -> noslip");
  F(con_b, "constraints -> noslip");
  F(tree_island, "islands -> finish"); F(isl_n, "islands -> finish"); F(isl_dof, "islands -> finish (union: xlo)");
  F(isl_eoff, "islands -> Newton"); F(isl_roff, "islands -> finish"); F(isl_joff, "islands -> finish");
  F(tree_ipos, "islands -> finish"); F(dof_ipos, "islands -> finish"); F(isl_row, "islands -> finish");
  F(isl_alpha, "Newton"); F(isl_cost, "Newton"); F(isl_val, "Newton"); F(isl_flag, "Newton"); F(isl_hvalid, "Newton");
  printf("\nlisted fields %zu B (union members overlap: the struct is %zu B)\n", tot, sizeof(E));
  printf("union pos: %zu B, union sol: %zu B, jt %zu, newton set %zu, noslip set %zu\n",
         offsetof(E, M) - offsetof(E, xpos), offsetof(E, M) - offsetof(E, jt), sizeof(((E*)0)->jt),
         sizeof(((E*)0)->Hp) + sizeof(((E*)0)->ntmp) + 2 * sizeof(((E*)0)->rr_f) + sizeof(((E*)0)->NL),
         sizeof(((E*)0)->efc_Wv) + sizeof(((E*)0)->ns_list) + sizeof(((E*)0)->ns_len) + sizeof(((E*)0)->rr_g));
  return 0;
}
