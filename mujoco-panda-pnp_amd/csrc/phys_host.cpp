// phys_host.cpp — builds the DevPhys<T> device image (phys_model.h) from pnp_model_desc.
//
// Host-side model compilation for the step kernel (the part of MuJoCo's compiler/mj_setConst
// the kernel relies on, plus the lane-parallel index tables).  Collision pair filtering follows
// MuJoCo 2.3.3 mj_collision: contype/conaffinity bitmask, same weld body (incl. static-static),
// weld parent/child when both are non-world (filterparent).  Pairs are kept in (g1 < g2) model
// order with g1 the lower geom type, the order the CPU oracle visits them.
#include <cstdio>
#include <cstring>

#include "phys_model.h"
#include "pnp_internal.h"

template <typename T>
int build_phys(const pnp_model_desc* s, DevPhys<T>* d, char* err, int errlen) {
  memset(d, 0, sizeof(*d));
  if (s->nbody > PH_MAXB || s->njnt > PH_MAXJ || s->nv > PH_MAXV || s->nq > PH_MAXQ || s->nu > PH_MAXU ||
      s->neq > 4 || s->nmocap > 2 || s->nbody > 32 || s->nv > 64 || s->nmesh > PH_MAXMESH ||
      s->nmeshvert > PH_MAXMESHV || s->nsite > PH_MAXS) {
    snprintf(err, errlen, "model exceeds the step kernel's compiled capacity");
    return -1;
  }
  // index consistency of the tables read below (a malformed description must not read past them)
  for (int k = 0; k < s->nmesh; k++)
    if (s->mesh_vertadr[k] < 0 || s->mesh_vertnum[k] < 0 || s->mesh_vertadr[k] + s->mesh_vertnum[k] > s->nmeshvert) {
      snprintf(err, errlen, "mesh %d: vertices [%d, %d) outside the %d mesh vertices", k, s->mesh_vertadr[k],
               s->mesh_vertadr[k] + s->mesh_vertnum[k], s->nmeshvert);
      return -1;
    }
  if (s->ngeom > 512) {   // (the collidable-geom map below)
    snprintf(err, errlen, "more than 512 geoms");
    return -1;
  }
  for (int g = 0; g < s->ngeom; g++)
    if (s->geom_bodyid[g] < 0 || s->geom_bodyid[g] >= s->nbody ||
        ((s->geom_contype[g] || s->geom_conaffinity[g]) && s->geom_type[g] == 7 &&
         (s->geom_dataid[g] < 0 || s->geom_dataid[g] >= s->nmesh))) {
      snprintf(err, errlen, "geom %d: body or mesh id out of range", g);
      return -1;
    }
  for (int b = 0; b < s->nbody; b++)
    if (s->body_parentid[b] < 0 || s->body_parentid[b] >= s->nbody || (b > 0 && s->body_parentid[b] >= b) ||
        s->body_jntadr[b] + s->body_jntnum[b] > s->njnt || s->body_dofadr[b] + s->body_dofnum[b] > s->nv) {
      snprintf(err, errlen, "body %d: parent / joint / dof ids out of range", b);
      return -1;
    }
  for (int j = 0; j < s->njnt; j++) {
    // qpos / dof widths of the joint type (mjtJoint: free 7 / 6, ball 4 / 3, slide and hinge 1 / 1)
    const int t = s->jnt_type[j];
    const int nqj = t == 0 ? 7 : (t == 1 ? 4 : 1), nvj = t == 0 ? 6 : (t == 1 ? 3 : 1);
    if (t < 0 || t > 3 || s->jnt_qposadr[j] < 0 || s->jnt_qposadr[j] + nqj > s->nq || s->jnt_dofadr[j] < 0 ||
        s->jnt_dofadr[j] + nvj > s->nv) {
      snprintf(err, errlen, "joint %d: qpos / dof address out of range", j);
      return -1;
    }
  }
  d->nq = s->nq; d->nv = s->nv; d->nu = s->nu; d->nbody = s->nbody; d->njnt = s->njnt;
  d->nmocap = s->nmocap; d->neq = s->neq;
  d->timestep = (T)s->timestep;
  for (int k = 0; k < 3; k++) d->gravity[k] = (T)s->gravity[k];
  d->noslip_iterations = s->noslip_iterations;
  d->iterations = s->iterations;
  d->tolerance = (T)s->tolerance;
  d->noslip_tolerance = (T)s->noslip_tolerance;
  d->meaninertia = (T)s->stat_meaninertia;
  if (!(s->stat_meaninertia > 0)) {
    snprintf(err, errlen, "stat_meaninertia must be > 0 (mj_setConst: mean of diag(M) at qpos0)");
    return -1;
  }
  d->multiccd = s->multiccd;
  // ---- bodies
  for (int b = 0; b < s->nbody; b++) {
    d->body_parentid[b] = s->body_parentid[b];
    d->body_rootid[b] = s->body_rootid[b];
    d->body_weldid[b] = s->body_weldid[b];
    d->body_mocapid[b] = s->body_mocapid[b];
    d->body_jntadr[b] = s->body_jntadr[b];
    d->body_jntnum[b] = s->body_jntnum[b];
    d->body_dofadr[b] = s->body_dofadr[b];
    d->body_dofnum[b] = s->body_dofnum[b];
    for (int k = 0; k < 3; k++) {
      d->body_pos[b][k] = (T)s->body_pos[3 * b + k];
      d->body_ipos[b][k] = (T)s->body_ipos[3 * b + k];
      d->body_inertia[b][k] = (T)s->body_inertia[3 * b + k];
    }
    for (int k = 0; k < 4; k++) {
      d->body_quat[b][k] = (T)s->body_quat[4 * b + k];
      d->body_iquat[b][k] = (T)s->body_iquat[4 * b + k];
    }
    d->body_mass[b] = (T)s->body_mass[b];
    d->body_invweight0[b][0] = (T)s->body_invweight0[2 * b];
    d->body_invweight0[b][1] = (T)s->body_invweight0[2 * b + 1];
    d->body_subtreemass[b] = (T)s->body_subtreemass[b];
    // root -> body path (world excluded)
    int path[PH_MAXDEPTH + 1], n = 0;
    for (int c = b; c > 0; c = s->body_parentid[c]) {
      if (n >= PH_MAXDEPTH) { snprintf(err, errlen, "tree deeper than %d", PH_MAXDEPTH); return -1; }
      path[n++] = c;
    }
    d->body_pathlen[b] = n;
    for (int k = 0; k < n; k++) d->body_path[b][k] = path[n - 1 - k];
    uint64_t dm = 0;
    for (int k = 0; k < n; k++) {
      int c = path[k];
      for (int q = 0; q < s->body_dofnum[c]; q++) dm |= 1ull << (s->body_dofadr[c] + q);
    }
    d->body_dofmask[b] = dm;
  }
  for (int b = 0; b < s->nbody; b++) {
    uint32_t st = 0;
    for (int c = 0; c < s->nbody; c++) {
      int x = c;
      while (x > 0 && x != b) x = s->body_parentid[x];
      if (x == b && (b > 0 || c == 0)) st |= 1u << c;
    }
    d->body_subtree[b] = st;
  }
  // ---- trees: root bodies (children of the world) whose subtree has dofs; dofs contiguous
  int ntree = 0;
  for (int b = 0; b < s->nbody; b++) d->body_tree[b] = -1;
  for (int r = 1; r < s->nbody; r++) {
    if (s->body_parentid[r] != 0) continue;
    int lo = 1 << 30, hi = -1;
    for (int c = 0; c < s->nbody; c++)
      if (d->body_subtree[r] >> c & 1)
        for (int q = 0; q < s->body_dofnum[c]; q++) {
          int dof = s->body_dofadr[c] + q;
          if (dof < lo) lo = dof;
          if (dof > hi) hi = dof;
        }
    if (hi < 0) continue;
    if (ntree >= PH_MAXT || hi - lo + 1 > PH_MAXTDOF) { snprintf(err, errlen, "too many trees / tree dofs"); return -1; }
    d->tree_dofadr[ntree] = lo;
    d->tree_dofnum[ntree] = hi - lo + 1;
    for (int c = 0; c < s->nbody; c++)
      if (d->body_subtree[r] >> c & 1) d->body_tree[c] = ntree;
    ntree++;
  }
  d->ntree = ntree;
  int moff = 0;
  for (int t = 0; t < ntree; t++) {
    d->tree_moff[t] = moff;
    moff += d->tree_dofnum[t] * d->tree_dofnum[t];
  }
  if (moff > PH_MAXMBLK) { snprintf(err, errlen, "tree mass-matrix blocks exceed capacity"); return -1; }
  d->nmblock = moff;
  // ---- joints
  for (int j = 0; j < s->njnt; j++) {
    d->jnt_type[j] = s->jnt_type[j];
    d->jnt_qposadr[j] = s->jnt_qposadr[j];
    d->jnt_dofadr[j] = s->jnt_dofadr[j];
    d->jnt_bodyid[j] = s->jnt_bodyid[j];
    d->jnt_limited[j] = s->jnt_limited[j];
    for (int k = 0; k < 3; k++) {
      d->jnt_pos[j][k] = (T)s->jnt_pos[3 * j + k];
      d->jnt_axis[j][k] = (T)s->jnt_axis[3 * j + k];
    }
    for (int k = 0; k < 2; k++) {
      d->jnt_range[j][k] = (T)s->jnt_range[2 * j + k];
      d->jnt_solref[j][k] = (T)s->jnt_solref[2 * j + k];
    }
    for (int k = 0; k < 5; k++) d->jnt_solimp[j][k] = (T)s->jnt_solimp[5 * j + k];
    d->jnt_margin[j] = (T)s->jnt_margin[j];
    if (s->jnt_type[j] == 1) { snprintf(err, errlen, "ball joints not supported by the step kernel"); return -1; }
  }
  // ---- dofs
  for (int i = 0; i < s->nv; i++) {
    d->dof_bodyid[i] = s->dof_bodyid[i];
    d->dof_jntid[i] = s->dof_jntid[i];
    d->dof_parentid[i] = s->dof_parentid[i];
    d->dof_tree[i] = d->body_tree[s->dof_bodyid[i]];
    d->dof_armature[i] = (T)s->dof_armature[i];
    d->dof_damping[i] = (T)s->dof_damping[i];
    d->dof_invweight0[i] = (T)s->dof_invweight0[i];
    // cvel used for cdof_dot: all strict ancestors; for the rotational dofs of a free joint the
    // ancestors of the joint plus its translational dofs (MuJoCo mj_comVel free/ball case)
    uint64_t vm = 0;
    int j = s->dof_jntid[i], first = s->jnt_dofadr[j];
    if (s->jnt_type[j] == 0 && i >= first + 3) {
      for (int a = s->dof_parentid[first]; a >= 0; a = s->dof_parentid[a]) vm |= 1ull << a;
      for (int q = 0; q < 3; q++) vm |= 1ull << (first + q);
    } else {
      for (int a = s->dof_parentid[i]; a >= 0; a = s->dof_parentid[a]) vm |= 1ull << a;
    }
    d->dof_velmask[i] = vm;
  }
  for (int i = 0; i < s->nq; i++) d->qpos0[i] = (T)s->qpos0[i];
  int ne = 0;
  for (int i = 0; i < s->nv; i++)
    for (int j = i; j >= 0; j = s->dof_parentid[j]) {
      if (ne >= PH_MAXMENTRY) { snprintf(err, errlen, "too many M entries"); return -1; }
      d->mentry_i[ne] = i;
      d->mentry_j[ne] = j;
      ne++;
    }
  d->nmentry = ne;
  // ---- collidable geoms + pairs
  int ng = 0, map[512];
  for (int g = 0; g < s->ngeom && g < 512; g++) {
    map[g] = -1;
    if (!s->geom_contype[g] && !s->geom_conaffinity[g]) continue;
    if (ng >= PH_MAXG) { snprintf(err, errlen, "too many collidable geoms"); return -1; }
    map[g] = ng;
    d->geom_id[ng] = g;
    d->geom_type[ng] = s->geom_type[g];
    d->geom_bodyid[ng] = s->geom_bodyid[g];
    d->geom_dataid[ng] = s->geom_dataid[g];
    d->geom_condim[ng] = s->geom_condim[g];
    d->geom_priority[ng] = s->geom_priority[g];
    for (int k = 0; k < 3; k++) {
      d->geom_size[ng][k] = (T)s->geom_size[3 * g + k];
      d->geom_pos[ng][k] = (T)s->geom_pos[3 * g + k];
      d->geom_friction[ng][k] = (T)s->geom_friction[3 * g + k];
    }
    for (int k = 0; k < 4; k++) d->geom_quat[ng][k] = (T)s->geom_quat[4 * g + k];
    for (int k = 0; k < 2; k++) d->geom_solref[ng][k] = (T)s->geom_solref[2 * g + k];
    for (int k = 0; k < 5; k++) d->geom_solimp[ng][k] = (T)s->geom_solimp[5 * g + k];
    d->geom_margin[ng] = (T)s->geom_margin[g];
    d->geom_gap[ng] = (T)s->geom_gap[g];
    d->geom_solmix[ng] = (T)s->geom_solmix[g];
    d->geom_rbound[ng] = (T)s->geom_rbound[g];
    {   // geom-frame bounding box (oracle/convex.c local_box)
      double c[3] = {0, 0, 0}, h[3] = {0, 0, 0};
      const int ty = s->geom_type[g];
      if (ty == 2) {
        h[0] = h[1] = h[2] = s->geom_size[3 * g];
      } else if (ty == 6) {
        for (int k = 0; k < 3; k++) h[k] = s->geom_size[3 * g + k];
      } else if (ty == 7 && s->geom_dataid[g] >= 0) {
        const int mesh = s->geom_dataid[g];
        const double* V = s->mesh_vert + 3 * s->mesh_vertadr[mesh];
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int i = 0; i < s->mesh_vertnum[mesh]; i++)
          for (int k = 0; k < 3; k++) {
            lo[k] = V[3 * i + k] < lo[k] ? V[3 * i + k] : lo[k];
            hi[k] = V[3 * i + k] > hi[k] ? V[3 * i + k] : hi[k];
          }
        for (int k = 0; k < 3; k++) { c[k] = 0.5 * (lo[k] + hi[k]); h[k] = 0.5 * (hi[k] - lo[k]); }
      }
      for (int k = 0; k < 3; k++) { d->geom_aabb[ng][k] = (T)c[k]; d->geom_aabb[ng][3 + k] = (T)h[k]; }
    }
    if (s->geom_type[g] != 0 && s->geom_type[g] != 2 && s->geom_type[g] != 6 && s->geom_type[g] != 7) {
      snprintf(err, errlen, "geom type %d not supported by the step kernel", s->geom_type[g]);
      return -1;
    }
    ng++;
  }
  d->ngeom = ng;
  int np = 0;
  for (int g1 = 0; g1 < s->ngeom; g1++) {
    if (map[g1] < 0) continue;
    for (int g2 = g1 + 1; g2 < s->ngeom; g2++) {
      if (map[g2] < 0) continue;
      int ct1 = s->geom_contype[g1], ca1 = s->geom_conaffinity[g1];
      int ct2 = s->geom_contype[g2], ca2 = s->geom_conaffinity[g2];
      if (!(ct1 & ca2) && !(ct2 & ca1)) continue;
      int w1 = s->body_weldid[s->geom_bodyid[g1]], w2 = s->body_weldid[s->geom_bodyid[g2]];
      if (w1 == w2) continue;
      int p1 = s->body_weldid[s->body_parentid[w1]], p2 = s->body_weldid[s->body_parentid[w2]];
      if (w1 != 0 && w2 != 0 && (w1 == p2 || w2 == p1)) continue;
      if (np >= PH_MAXPAIR) { snprintf(err, errlen, "too many collision pairs"); return -1; }
      int a = g1, b = g2;
      if (s->geom_type[a] > s->geom_type[b]) { int t = a; a = b; b = t; }
      d->pair_g1[np] = map[a];
      d->pair_g2[np] = map[b];
      const double ra = s->geom_rbound[a], rb = s->geom_rbound[b];
      const double mg = s->geom_margin[a] > s->geom_margin[b] ? s->geom_margin[a] : s->geom_margin[b];
      d->pair_reach[np] = (T)(ra > 0 && rb > 0 ? ra + rb + mg : -1.0);
      d->pair_margin[np] = (T)mg;
      const int ta = s->geom_type[a], tb = s->geom_type[b];
      d->pair_kind[np] = tb == 7 && ta != 0 ? PH_PAIR_CONVEX
                         : ta == 0 && tb != 0 ? PH_PAIR_PLANE
                         : ta == 6 && tb == 6 ? PH_PAIR_BOX : PH_PAIR_PRIM;
      np++;
    }
  }
  d->npair = np;
  // ---- body-pair pre-cull (result-neutral: a body sphere contains its geoms' spheres)
  {
    const double slack = 1e-5;
    for (int b = 0; b < s->nbody; b++) {
      double c[3] = {0, 0, 0}, lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
      int cnt = 0, plane = 0;
      for (int g = 0; g < s->ngeom; g++) {
        if (map[g] < 0 || s->geom_bodyid[g] != b) continue;
        if (!(s->geom_rbound[g] > 0)) { plane = 1; continue; }
        for (int k = 0; k < 3; k++) {
          const double v = s->geom_pos[3 * g + k];
          lo[k] = v - s->geom_rbound[g] < lo[k] ? v - s->geom_rbound[g] : lo[k];
          hi[k] = v + s->geom_rbound[g] > hi[k] ? v + s->geom_rbound[g] : hi[k];
        }
        cnt++;
      }
      double r = 0;
      if (cnt) {
        for (int k = 0; k < 3; k++) c[k] = 0.5 * (lo[k] + hi[k]);
        for (int g = 0; g < s->ngeom; g++) {
          if (map[g] < 0 || s->geom_bodyid[g] != b || !(s->geom_rbound[g] > 0)) continue;
          double dd = 0;
          for (int k = 0; k < 3; k++) dd += (s->geom_pos[3 * g + k] - c[k]) * (s->geom_pos[3 * g + k] - c[k]);
          const double rr = __builtin_sqrt(dd) + s->geom_rbound[g];
          r = rr > r ? rr : r;
        }
      }
      for (int k = 0; k < 3; k++) d->body_bcen[b][k] = (T)c[k];
      d->body_brad[b] = plane ? (T)-1 : (T)(r * (1 + slack) + slack);
    }
    int nbp = 0;
    static thread_local int grp[PH_MAXPAIR];
    for (int p = 0; p < np; p++) grp[p] = -1;
    for (int p = 0; p < np; p++) {
      if (grp[p] >= 0) continue;
      if (nbp >= PH_MAXBP) { snprintf(err, errlen, "too many collision body pairs"); return -1; }
      const int g1 = d->geom_id[d->pair_g1[p]], g2 = d->geom_id[d->pair_g2[p]];
      int b1 = s->geom_bodyid[g1], b2 = s->geom_bodyid[g2];
      if (b1 > b2) { const int t = b1; b1 = b2; b2 = t; }
      d->bp_b1[nbp] = (short)b1;
      d->bp_b2[nbp] = (short)b2;
      double mg = 0;
      for (int q = p; q < np; q++) {
        const int h1 = d->geom_id[d->pair_g1[q]], h2 = d->geom_id[d->pair_g2[q]];
        int c1 = s->geom_bodyid[h1], c2 = s->geom_bodyid[h2];
        if (c1 > c2) { const int t = c1; c1 = c2; c2 = t; }
        if (c1 != b1 || c2 != b2) continue;
        grp[q] = nbp;
        mg = (double)d->pair_margin[q] > mg ? (double)d->pair_margin[q] : mg;
      }
      const double r1 = (double)d->body_brad[b1], r2 = (double)d->body_brad[b2];
      d->bp_reach[nbp] = (T)(r1 < 0 || r2 < 0 ? -1.0 : (r1 + r2 + mg) * (1 + slack) + slack);
      nbp++;
    }
    d->nbpair = nbp;
    for (int p = 0; p < np; p++)
      d->pair_pack[p] = (uint32_t)d->pair_g1[p] | (uint32_t)d->pair_g2[p] << 8 |
                        (uint32_t)d->pair_kind[p] << 16 | (uint32_t)grp[p] << 24;
  }
  for (int k = 0; k < s->nmesh; k++) {
    d->mesh_vertadr[k] = s->mesh_vertadr[k];
    d->mesh_vertnum[k] = s->mesh_vertnum[k];
  }
  for (int v = 0; v < s->nmeshvert; v++)
    for (int k = 0; k < 3; k++) d->mesh_vert[v][k] = (T)s->mesh_vert[3 * v + k];
  // ---- actuators
  for (int i = 0; i < s->nu; i++) {
    int j = s->actuator_trnid[i];
    d->act_trnid[i] = j;
    d->act_dof[i] = s->jnt_dofadr[j];
    d->act_qadr[i] = s->jnt_qposadr[j];
    d->act_biastype[i] = s->actuator_biastype[i];
    d->act_ctrllimited[i] = s->actuator_ctrllimited[i];
    d->act_forcelimited[i] = s->actuator_forcelimited[i];
    d->act_gear[i] = (T)s->actuator_gear[i];
    for (int k = 0; k < 3; k++) {
      d->act_gainprm[i][k] = (T)s->actuator_gainprm[3 * i + k];
      d->act_biasprm[i][k] = (T)s->actuator_biasprm[3 * i + k];
    }
    for (int k = 0; k < 2; k++) {
      d->act_ctrlrange[i][k] = (T)s->actuator_ctrlrange[2 * i + k];
      d->act_forcerange[i][k] = (T)s->actuator_forcerange[2 * i + k];
    }
  }
  for (int d0 = 0; d0 < PH_MAXV; d0++) d->dof_act[d0] = -1;
  for (int i = 0; i < s->nu; i++) {
    int& da = d->dof_act[d->act_dof[i]];
    da = da == -1 ? i : -2;
  }
  // ---- equality
  for (int e = 0; e < s->neq; e++) {
    d->eq_type[e] = s->eq_type[e];
    d->eq_obj1id[e] = s->eq_obj1id[e];
    d->eq_obj2id[e] = s->eq_obj2id[e];
    for (int k = 0; k < 2; k++) d->eq_solref[e][k] = (T)s->eq_solref[2 * e + k];
    for (int k = 0; k < 5; k++) d->eq_solimp[e][k] = (T)s->eq_solimp[5 * e + k];
    for (int k = 0; k < 11; k++) d->eq_data[e][k] = (T)s->eq_data[11 * e + k];
  }
  for (int b = 0; b < s->nbody; b++)
    if (s->body_mocapid[b] >= 0) d->mocap_body[s->body_mocapid[b]] = b;
  // ---- fp64 chain constants + the first weld (see DevPhys::kd_*)
  d->weld_eq = -1;
  d->weld_body[0] = d->weld_body[1] = -1;
  for (int e = 0; e < s->neq && d->weld_eq < 0; e++)
    if (s->eq_type[e] == 1) {
      d->weld_eq = e;
      d->weld_body[0] = s->eq_obj1id[e];
      d->weld_body[1] = s->eq_obj2id[e];
      for (int k = 0; k < 11; k++) d->kd_eq_data[k] = s->eq_data[11 * e + k];
    }
  for (int b = 0; b < s->nbody; b++) {
    for (int k = 0; k < 3; k++) d->kd_body_pos[b][k] = s->body_pos[3 * b + k];
    for (int k = 0; k < 4; k++) d->kd_body_quat[b][k] = s->body_quat[4 * b + k];
    const int j = s->body_jntadr[b];
    const bool one = s->body_jntnum[b] == 1;
    for (int k = 0; k < 3; k++) {
      d->kd_jnt_pos[b][k] = one ? s->jnt_pos[3 * j + k] : 0.0;
      d->kd_jnt_axis[b][k] = one ? s->jnt_axis[3 * j + k] : 0.0;
    }
    d->kd_qpos0[b] = one && s->jnt_type[j] != 0 ? s->qpos0[s->jnt_qposadr[j]] : 0.0;
  }
  // ---- sites
  d->nsite = s->nsite;
  for (int i = 0; i < s->nsite; i++) {
    d->site_bodyid[i] = s->site_bodyid[i];
    for (int k = 0; k < 3; k++) d->site_pos[i][k] = (T)s->site_pos[3 * i + k];
    for (int k = 0; k < 4; k++) d->site_quat[i][k] = (T)s->site_quat[4 * i + k];
  }
  return 0;
}

template int build_phys<float>(const pnp_model_desc*, DevPhys<float>*, char*, int);
template int build_phys<double>(const pnp_model_desc*, DevPhys<double>*, char*, int);
