/*
 * collision.c — mj_collision restated (MuJoCo 2.3.3 engine_collision_driver.c, _primitive.c,
 * _box.c, _convex.c).  TEST INFRASTRUCTURE ONLY (see oracle.c).
 *
 * Broadphase: every pair of collidable geoms (contype/conaffinity bitmask test), skipping pairs
 * on the same weld body (incl. static-static) and weld parent/child pairs when both are
 * non-world (filterparent); bounding-sphere test with margin.  This visits a superset of what
 * MuJoCo's sweep-and-prune visits; the extra pairs are disjoint and produce no contact.
 * Narrowphase by type (geom1 has the lower type; same type: lower geom id first), contact
 * normal from geom1 to geom2, contact position midway between the surfaces:
 *   plane-sphere, plane-box (corners below the plane, deepest-first as MuJoCo, <= 4),
 *   plane-mesh (hull vertices below the plane, <= 4 deepest), sphere-sphere, sphere-box,
 *   box-box (separating-axis test over 15 axes, reference/incident face clipping, edge-edge),
 *   convex mesh pairs (mesh-*): convex.c.
 * Contact parameters (mj_contactParam): condim and friction = max, solref/solimp mixed by
 * solmix, margin/gap = max.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "physics.h"
#include "spatial.h"

typedef const pnp_model_desc Mdl;

enum { T_PLANE = 0, T_SPHERE = 2, T_BOX = 6, T_MESH = 7 };

int orc_convex_collide(Mdl* m, const orc_data* d, int g1, int g2, double margin, orc_contact* out, int cap);

static int geom_filter_skip(Mdl* m, int g1, int g2) {
  int ct1 = m->geom_contype[g1], ca1 = m->geom_conaffinity[g1];
  int ct2 = m->geom_contype[g2], ca2 = m->geom_conaffinity[g2];
  if (!(ct1 & ca2) && !(ct2 & ca1)) return 1;
  int w1 = m->body_weldid[m->geom_bodyid[g1]], w2 = m->body_weldid[m->geom_bodyid[g2]];
  if (w1 == w2) return 1;
  int p1 = m->body_weldid[m->body_parentid[w1]], p2 = m->body_weldid[m->body_parentid[w2]];
  if (w1 != 0 && w2 != 0 && (w1 == p2 || w2 == p1)) return 1;
  return 0;
}

static void set_normal(orc_contact* c, const double n[3]) {
  memset(c->frame, 0, sizeof(c->frame));
  c->frame[0] = n[0]; c->frame[1] = n[1]; c->frame[2] = n[2];
}

/* ---------------------------------------------------------------- primitive colliders */
static int plane_sphere(const double* p1, const double* R1, const double* p2, double r, double margin,
                        orc_contact* c) {
  double n[3] = {R1[2], R1[5], R1[8]}, v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double dist = dot3(v, n) - r;
  if (dist > margin) return 0;
  c->dist = dist;
  set_normal(c, n);
  for (int k = 0; k < 3; k++) c->pos[k] = p2[k] - n[k] * (r + dist * 0.5);
  return 1;
}

static int plane_box(const double* p1, const double* R1, const double* p2, const double* R2,
                     const double* s, double margin, orc_contact* c) {
  double n[3] = {R1[2], R1[5], R1[8]}, v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double dist = dot3(v, n);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double cr[3] = {(i & 1) ? s[0] : -s[0], (i & 2) ? s[1] : -s[1], (i & 4) ? s[2] : -s[2]}, w[3];
    mulmatvec3(w, R2, cr);
    double ld = dot3(n, w);
    if (dist + ld > margin || ld > 0) continue;
    c[cnt].dist = dist + ld;
    set_normal(c + cnt, n);
    for (int k = 0; k < 3; k++) c[cnt].pos[k] = w[k] + p2[k] - n[k] * c[cnt].dist * 0.5;
    if (++cnt >= 4) return 4;
  }
  return cnt;
}

static int plane_mesh(Mdl* m, const double* p1, const double* R1, const double* p2, const double* R2,
                      int mesh, double margin, orc_contact* c) {
  double n[3] = {R1[2], R1[5], R1[8]};
  const double* V = m->mesh_vert + 3 * m->mesh_vertadr[mesh];
  int nvert = m->mesh_vertnum[mesh];
  double best[4]; int bi[4], cnt = 0;
  for (int i = 0; i < nvert; i++) {
    double w[3];
    mulmatvec3(w, R2, V + 3 * i);
    double dd = (w[0] + p2[0] - p1[0]) * n[0] + (w[1] + p2[1] - p1[1]) * n[1] + (w[2] + p2[2] - p1[2]) * n[2];
    if (dd > margin) continue;
    /* keep the 4 deepest (ties: lower vertex index) */
    int pos = cnt < 4 ? cnt : 4;
    while (pos > 0 && best[pos - 1] > dd) pos--;
    if (pos >= 4) continue;
    for (int k = (cnt < 4 ? cnt : 3); k > pos; k--) { best[k] = best[k - 1]; bi[k] = bi[k - 1]; }
    best[pos] = dd; bi[pos] = i;
    if (cnt < 4) cnt++;
  }
  for (int k = 0; k < cnt; k++) {
    double w[3];
    mulmatvec3(w, R2, V + 3 * bi[k]);
    c[k].dist = best[k];
    set_normal(c + k, n);
    for (int t = 0; t < 3; t++) c[k].pos[t] = w[t] + p2[t] - n[t] * best[k] * 0.5;
  }
  return cnt;
}

static int sphere_sphere(const double* p1, double r1, const double* p2, double r2, double margin,
                         orc_contact* c) {
  double n[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double len = sqrt(dot3(n, n));
  double dist = len - r1 - r2;
  if (dist > margin) return 0;
  if (len < ORC_MINVAL) { n[0] = 1; n[1] = 0; n[2] = 0; }
  else { n[0] /= len; n[1] /= len; n[2] /= len; }
  c->dist = dist;
  set_normal(c, n);
  for (int k = 0; k < 3; k++) c->pos[k] = p1[k] + n[k] * (r1 + dist * 0.5);
  return 1;
}

static int sphere_box(const double* p1, double r, const double* p2, const double* R2, const double* s,
                      double margin, orc_contact* c) {
  double v[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]}, lc[3], cl[3], nl[3], n[3];
  mulmattvec3(lc, R2, v);
  int inside = 1;
  for (int k = 0; k < 3; k++) {
    cl[k] = fmin(fmax(lc[k], -s[k]), s[k]);
    if (cl[k] != lc[k]) inside = 0;
  }
  double dist;
  if (!inside) {
    for (int k = 0; k < 3; k++) nl[k] = cl[k] - lc[k];
    double dd = sqrt(dot3(nl, nl));
    dist = dd - r;
    if (dist > margin) return 0;
    for (int k = 0; k < 3; k++) nl[k] /= dd;
  } else {
    int kk = 0;
    double pen = s[0] - fabs(lc[0]);
    for (int k = 1; k < 3; k++)
      if (s[k] - fabs(lc[k]) < pen) { pen = s[k] - fabs(lc[k]); kk = k; }
    nl[0] = nl[1] = nl[2] = 0;
    nl[kk] = lc[kk] >= 0 ? -1 : 1;
    dist = -(pen + r);
  }
  mulmatvec3(n, R2, nl);
  c->dist = dist;
  set_normal(c, n);
  for (int k = 0; k < 3; k++) c->pos[k] = p1[k] + n[k] * (r + dist * 0.5);
  return 1;
}

/* 1 um band that moves box-box decisions off exact configurations: identical boxes pressed face
 * to face (the closed gripper's finger pads) put every clip / corner / SAT-tie / inclusion test
 * exactly on its boundary, where rounding (FMA or not) would decide.  Applied identically by
 * the device colliders. */
#define BB_TOL 1e-6

/* Liang-Barsky: clip the 2D segment p0 -> p1 (x, y = coords 0, 1) to |x| <= A, |y| <= B (closed);
 * returns 0 when nothing is left, else the parameter interval [t0, t1] */
static int clip_seg(const double* p0, const double* p1, double A, double B, double* t0, double* t1) {
  const double dx = p1[0] - p0[0], dy = p1[1] - p0[1];
  const double pp[4] = {-dx, dx, -dy, dy}, qq[4] = {p0[0] + A, A - p0[0], p0[1] + B, B - p0[1]};
  double a = 0, b = 1;
  for (int k = 0; k < 4; k++) {
    if (pp[k] == 0) {
      if (qq[k] < 0) return 0;
    } else {
      const double r = qq[k] / pp[k];
      if (pp[k] < 0) { if (r > a) a = r; } else { if (r < b) b = r; }
    }
  }
  if (a > b) return 0;
  *t0 = a;
  *t1 = b;
  return 1;
}

/* Reference face on box r (axis ia, outward normal nr), incident box i; nframe = contact normal.
 * The incident face (the face of box i most anti-parallel to nr) is expressed in the reference
 * face frame (u, v, depth along nr) and intersected with the reference rectangle.  The vertices
 * of that convex polygon are emitted in a fixed order: for each incident edge e = 0..3 its clipped
 * start point and, when the edge leaves the rectangle, its exit point; then the reference corners
 * strictly inside the incident face (depth from the incident plane).  This is the vertex set
 * reference-face clipping (Sutherland-Hodgman) produces, computed without a variable-length
 * polygon so the device version stays in registers; points deeper than margin are dropped.
 * Not MuJoCo's mjc_BoxBox contact reduction: parity with MuJoCo here is unpinned. */
static int box_face_contacts(const double* pr, const double* Rr, const double* sr, int ia, const double* nr,
                             const double* pi, const double* Ri, const double* si, const double* nframe,
                             double margin, orc_contact* c) {
  int iu = (ia + 1) % 3, iv = (ia + 2) % 3;
  double u[3] = {Rr[iu], Rr[3 + iu], Rr[6 + iu]}, v[3] = {Rr[iv], Rr[3 + iv], Rr[6 + iv]};
  double cref[3];
  for (int k = 0; k < 3; k++) cref[k] = pr[k] + nr[k] * sr[ia];
  int ja = 0;
  double best = -1;
  for (int j = 0; j < 3; j++) {
    double a = fabs(Ri[j] * nr[0] + Ri[3 + j] * nr[1] + Ri[6 + j] * nr[2]);
    if (a > best) { best = a; ja = j; }
  }
  double bj[3] = {Ri[ja], Ri[3 + ja], Ri[6 + ja]};
  double sg = dot3(bj, nr) > 0 ? -1 : 1;
  int ju = (ja + 1) % 3, jv = (ja + 2) % 3;
  double bu[3] = {Ri[ju], Ri[3 + ju], Ri[6 + ju]}, bv[3] = {Ri[jv], Ri[3 + jv], Ri[6 + jv]};
  static const double su[4] = {1, -1, -1, 1}, sv[4] = {1, 1, -1, -1};
  double P[4][3];
  for (int q = 0; q < 4; q++) {
    double w[3];
    for (int k = 0; k < 3; k++) w[k] = pi[k] + sg * bj[k] * si[ja] + su[q] * bu[k] * si[ju] + sv[q] * bv[k] * si[jv] - cref[k];
    P[q][0] = dot3(w, u); P[q][1] = dot3(w, v); P[q][2] = dot3(w, nr);
  }
  const double A = sr[iu] + BB_TOL, B = sr[iv] + BB_TOL;   /* rectangle grown by the band */
  double pts[12][3];
  int np = 0;
  for (int e = 0; e < 4; e++) {
    const double* p0 = P[e];
    const double* p1 = P[(e + 1) & 3];
    double t0, t1;
    if (!clip_seg(p0, p1, A, B, &t0, &t1)) continue;
    for (int k = 0; k < 3; k++) pts[np][k] = p0[k] + t0 * (p1[k] - p0[k]);
    np++;
    if (t1 < 1) {
      for (int k = 0; k < 3; k++) pts[np][k] = p0[k] + t1 * (p1[k] - p0[k]);
      np++;
    }
  }
  /* reference corners inside the incident parallelogram P0 + a (P1 - P0) + b (P3 - P0) */
  const double e1[3] = {P[1][0] - P[0][0], P[1][1] - P[0][1], P[1][2] - P[0][2]};
  const double e3[3] = {P[3][0] - P[0][0], P[3][1] - P[0][1], P[3][2] - P[0][2]};
  const double det = e1[0] * e3[1] - e1[1] * e3[0];
  if (fabs(det) > 1e-12 * (fabs(e1[0]) + fabs(e1[1])) * (fabs(e3[0]) + fabs(e3[1]))) {
    /* corners more than the band inside the incident face (in its edge coordinates) */
    const double ta = BB_TOL / sqrt(e1[0] * e1[0] + e1[1] * e1[1]), tb = BB_TOL / sqrt(e3[0] * e3[0] + e3[1] * e3[1]);
    for (int q = 0; q < 4; q++) {
      const double cx = su[q] * sr[iu] - P[0][0], cy = sv[q] * sr[iv] - P[0][1];
      const double al = (cx * e3[1] - cy * e3[0]) / det, be = (e1[0] * cy - e1[1] * cx) / det;
      if (al > ta && al < 1 - ta && be > tb && be < 1 - tb) {
        pts[np][0] = su[q] * sr[iu];
        pts[np][1] = sv[q] * sr[iv];
        pts[np][2] = P[0][2] + al * e1[2] + be * e3[2];
        np++;
      }
    }
  }
  int cnt = 0;
  for (int q = 0; q < np && cnt < 8; q++) {
    double dist = pts[q][2];
    if (dist > margin + BB_TOL) continue;
    c[cnt].dist = dist;
    set_normal(c + cnt, nframe);
    for (int k = 0; k < 3; k++)
      c[cnt].pos[k] = cref[k] + u[k] * pts[q][0] + v[k] * pts[q][1] + nr[k] * pts[q][2] * 0.5;
    cnt++;
  }
  return cnt;
}

/* Box-box (MuJoCo 2.3.3 engine_collision_box.c mjc_BoxBox -- absent here; what follows is a
 * separating-axis restatement, and each point where it may differ from MuJoCo's routine is an
 * assumption, unverified, listed so a reader with the source can check them one by one):
 *   A1. Axes: the 15 SAT axes -- box 1's face normals, box 2's, then the 9 edge cross products
 *       A_i x B_j (skipped when |A_i x B_j| < 1e-6: parallel edges add nothing a face axis lacks).
 *   A2. Separation on any axis beyond the margin: no contact (the pair's early exit).
 *   A3. The contact axis is the one of least penetration, with ties and near-ties resolved toward
 *       faces: box 2's face replaces box 1's only when deeper by more than BB_TOL, and an edge axis
 *       wins only when 1.05 x its separation still beats the best face's by more than BB_TOL (ODE's
 *       dBoxBox uses the same 1.05 edge fudge factor; MuJoCo's exact bias is assumed, not known).
 *       The absolute BB_TOL matters where the factor cannot: two parallel boxes touching face to
 *       face at distance ~0 (the closed gripper's finger pads) have an edge axis A_i x B_j equal to
 *       the face normal with the same separation, and 1.05 x 0 decides nothing -- rounding picked
 *       the edge axis (one contact) in one arithmetic and the face (the clipped rectangle's four)
 *       in another (round 5 had a 1e-12 margin: the fp32 kernel made 1 contact per pad pair where
 *       the oracle made 4, tools/knife_edge_pairs.py).
 *   A4. Face axis: the incident face of the other box (the face most anti-parallel to the contact
 *       normal) is clipped against the reference face's rectangle (grown by BB_TOL); the contacts
 *       are the clipped polygon's vertices -- incident edge entry / exit points in edge order, then
 *       the reference corners inside the incident face -- at most 8, each with its own depth along
 *       the normal, kept when that depth is within the margin.  MuJoCo may reduce the polygon to
 *       fewer points (a known difference of contact COUNT on tilted faces, not on a box resting
 *       flat, where every routine yields the four corners of the contact face).
 *   A5. Contact position: halfway between the two surfaces along the normal (MuJoCo's convention
 *       for every primitive pair), normal from box 1 to box 2, dist = -penetration.
 *   A6. Edge axis: one contact at the midpoint of the two edges' closest points, depth = the axis
 *       separation.
 * Pinned without MuJoCo by geometric known answers (tests/test_boxbox_cpu.py: a cube resting flat,
 * tilted onto an edge and onto a corner, two cubes crossing edge to edge, deep spawns inside a shelf
 * or table leg and inside another cube -- the contact points and depths any correct box-box routine
 * must produce there) and by the reference's behavioural tests (grasp, lift, placement).  The
 * device colliders (collide_dev.h c_box_box / c_box_face) are this routine in box-relative
 * coordinates, equal to it at 1e-9 in fp64 (tests/test_boxbox_gpu.py). */
/* Assumption probes (tools/badqacc_probe.py; default 0 = the restatement above): bits that change
 * one assumption each, to test which of them, changed, could produce MUJOCO_LOG.TXT's BADQACC.
 *   1  A1: near-parallel edge axes kept down to |A_i x B_j| > 1e-12 (not 1e-6)
 *   2  A3: round 5's edge tie margin (1e-12 instead of BB_TOL)
 *   4  A6: no parallel-line guard on the edge closest points (den > 0, not den > 1e-12)
 *   8  A6: the edge contact at box 2's closest point (MuJoCo may place it on one edge) */
static int g_bb_variant = 0;
void orc_set_boxbox_variant(int v) { g_bb_variant = v; }
static int box_box(const double* p1, const double* R1, const double* s1, const double* p2, const double* R2,
                   const double* s2, double margin, orc_contact* c) {
  double T[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double A[3][3], B[3][3], AB[3][3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = R1[3 * k + i]; B[i][k] = R2[3 * k + i]; }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) AB[i][j] = dot3(A[i], B[j]);
  double best = -1e300, bestn[3] = {0, 0, 0};
  int btype = -1, bi = 0, bj = 0;
  for (int i = 0; i < 3; i++) {
    double tl = dot3(T, A[i]);
    double rb = s2[0] * fabs(AB[i][0]) + s2[1] * fabs(AB[i][1]) + s2[2] * fabs(AB[i][2]);
    double sep = fabs(tl) - s1[i] - rb;
    if (sep > margin) return 0;
    if (sep > best) { best = sep; btype = 0; bi = i; for (int k = 0; k < 3; k++) bestn[k] = tl >= 0 ? A[i][k] : -A[i][k]; }
  }
  for (int j = 0; j < 3; j++) {
    double tl = dot3(T, B[j]);
    double ra = s1[0] * fabs(AB[0][j]) + s1[1] * fabs(AB[1][j]) + s1[2] * fabs(AB[2][j]);
    double sep = fabs(tl) - ra - s2[j];
    if (sep > margin) return 0;
    /* box 2's faces replace box 1's only when clearly better (ties: identical boxes face to face) */
    if (sep > best + BB_TOL) { best = sep; btype = 1; bj = j; for (int k = 0; k < 3; k++) bestn[k] = tl >= 0 ? B[j][k] : -B[j][k]; }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double L[3];
      cross3(L, A[i], B[j]);
      double len = sqrt(dot3(L, L));
      if (len < ((g_bb_variant & 1) ? 1e-12 : 1e-6)) continue;
      for (int k = 0; k < 3; k++) L[k] /= len;
      double tl = dot3(T, L);
      double ra = s1[0] * fabs(dot3(A[0], L)) + s1[1] * fabs(dot3(A[1], L)) + s1[2] * fabs(dot3(A[2], L));
      double rb = s2[0] * fabs(dot3(B[0], L)) + s2[1] * fabs(dot3(B[1], L)) + s2[2] * fabs(dot3(B[2], L));
      double sep = fabs(tl) - ra - rb;
      if (sep > margin) return 0;
      /* edge axes must beat face axes clearly (ODE-style 1.05 depth fudge, and by BB_TOL: A3) */
      if (1.05 * sep > best + ((g_bb_variant & 2) ? 1e-12 : BB_TOL)) {
        best = sep; btype = 2; bi = i; bj = j;
        for (int k = 0; k < 3; k++) bestn[k] = tl >= 0 ? L[k] : -L[k];
      }
    }
  if (btype == 0) return box_face_contacts(p1, R1, s1, bi, bestn, p2, R2, s2, bestn, margin, c);
  if (btype == 1) {
    double nr[3] = {-bestn[0], -bestn[1], -bestn[2]};
    return box_face_contacts(p2, R2, s2, bj, nr, p1, R1, s1, bestn, margin, c);
  }
  /* edge-edge: closest points of the two supporting edges */
  double pa[3], pb[3];
  for (int k = 0; k < 3; k++) { pa[k] = p1[k]; pb[k] = p2[k]; }
  for (int t = 0; t < 3; t++) {
    if (t != bi) {
      double sg = dot3(A[t], bestn) > 0 ? 1 : -1;
      for (int k = 0; k < 3; k++) pa[k] += sg * s1[t] * A[t][k];
    }
    if (t != bj) {
      double sg = dot3(B[t], bestn) > 0 ? -1 : 1;
      for (int k = 0; k < 3; k++) pb[k] += sg * s2[t] * B[t][k];
    }
  }
  double ua[3] = {A[bi][0], A[bi][1], A[bi][2]}, ub[3] = {B[bj][0], B[bj][1], B[bj][2]};
  double w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
  double a = dot3(ua, ub), dd = dot3(ua, w), e = dot3(ub, w), den = 1 - a * a;
  double ta = 0, tb = 0;
  if (den > ((g_bb_variant & 4) ? 0.0 : 1e-12)) { ta = (a * e - dd) / den; tb = (e - a * dd) / den; }
  for (int k = 0; k < 3; k++) { pa[k] += ta * ua[k]; pb[k] += tb * ub[k]; }
  c->dist = best;
  set_normal(c, bestn);
  for (int k = 0; k < 3; k++) c->pos[k] = (g_bb_variant & 8) ? pb[k] : 0.5 * (pa[k] + pb[k]);
  return 1;
}

/* ---------------------------------------------------------------- contact parameters */
static void contact_params(Mdl* m, orc_contact* c, int g1, int g2) {
  c->geom1 = g1;
  c->geom2 = g2;
  c->dim = m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
  if (m->geom_priority[g1] != m->geom_priority[g2]) {
    int gp = m->geom_priority[g1] > m->geom_priority[g2] ? g1 : g2;
    c->dim = m->geom_condim[gp];
  }
  double f[3];
  for (int k = 0; k < 3; k++) f[k] = fmax(m->geom_friction[3 * g1 + k], m->geom_friction[3 * g2 + k]);
  c->friction[0] = c->friction[1] = f[0];
  c->friction[2] = f[1];
  c->friction[3] = c->friction[4] = f[2];
  double s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2], mix;
  if (s1 >= ORC_MINVAL && s2 >= ORC_MINVAL) mix = s1 / (s1 + s2);
  else if (s1 < ORC_MINVAL && s2 < ORC_MINVAL) mix = 0.5;
  else mix = s1 < ORC_MINVAL ? 0 : 1;
  const double *r1 = m->geom_solref + 2 * g1, *r2 = m->geom_solref + 2 * g2;
  if (r1[0] > 0 && r2[0] > 0) for (int k = 0; k < 2; k++) c->solref[k] = mix * r1[k] + (1 - mix) * r2[k];
  else for (int k = 0; k < 2; k++) c->solref[k] = fmin(r1[k], r2[k]);
  for (int k = 0; k < 5; k++) c->solimp[k] = mix * m->geom_solimp[5 * g1 + k] + (1 - mix) * m->geom_solimp[5 * g2 + k];
  double margin = fmax(m->geom_margin[g1], m->geom_margin[g2]);
  double gap = fmax(m->geom_gap[g1], m->geom_gap[g2]);
  c->includemargin = margin - gap;
}

int orc_collide_pair(Mdl* m, const orc_data* d, int g1, int g2, orc_contact* out, int cap) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  if (t1 > t2 || (t1 == t2 && g1 > g2)) { int t = g1; g1 = g2; g2 = t; t = t1; t1 = t2; t2 = t; }
  const double *p1 = d->geom_xpos + 3 * g1, *R1 = d->geom_xmat + 9 * g1, *s1 = m->geom_size + 3 * g1;
  const double *p2 = d->geom_xpos + 3 * g2, *R2 = d->geom_xmat + 9 * g2, *s2 = m->geom_size + 3 * g2;
  double margin = fmax(m->geom_margin[g1], m->geom_margin[g2]);
  orc_contact tmp[8];
  int n = 0;
  if (t1 == T_PLANE && t2 == T_SPHERE) n = plane_sphere(p1, R1, p2, s2[0], margin, tmp);
  else if (t1 == T_PLANE && t2 == T_BOX) n = plane_box(p1, R1, p2, R2, s2, margin, tmp);
  else if (t1 == T_PLANE && t2 == T_MESH) n = plane_mesh(m, p1, R1, p2, R2, m->geom_dataid[g2], margin, tmp);
  else if (t1 == T_SPHERE && t2 == T_SPHERE) n = sphere_sphere(p1, s1[0], p2, s2[0], margin, tmp);
  else if (t1 == T_SPHERE && t2 == T_BOX) n = sphere_box(p1, s1[0], p2, R2, s2, margin, tmp);
  else if (t1 == T_BOX && t2 == T_BOX) n = box_box(p1, R1, s1, p2, R2, s2, margin, tmp);
  else if (t2 == T_MESH && t1 != T_PLANE) n = orc_convex_collide(m, d, g1, g2, margin, tmp, 8);
  if (n > cap) n = cap;
  for (int k = 0; k < n; k++) {
    out[k] = tmp[k];
    /* colliders set the normal only; complete the tangent frame (mju_makeFrame, as
       mj_collideGeoms does before the contact enters the constraint Jacobian) */
    sp_makeframe(out[k].frame);
    contact_params(m, out + k, g1, g2);
  }
  return n;
}

/* convex (MPR) pair: (sphere | box | mesh) x mesh */
static int is_convex_pair(Mdl* m, int g1, int g2) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  int lo = t1 < t2 ? t1 : t2, hi = t1 < t2 ? t2 : t1;
  return hi == T_MESH && lo != T_PLANE;
}

/* Contact order: the primitive pairs in pair order, then the convex (MPR) pairs in pair order
 * (MuJoCo's order follows its sweep-and-prune output, not geom ids; this is the order the
 * device kernel produces, and the Gauss-Seidel noslip sweep depends on it). */
int orc_collision(Mdl* m, orc_data* d) {
  d->ncon = 0;
  for (int pass = 0; pass < 2; pass++)
    for (int g1 = 0; g1 < m->ngeom; g1++) {
      if (!m->geom_contype[g1] && !m->geom_conaffinity[g1]) continue;
      for (int g2 = g1 + 1; g2 < m->ngeom; g2++) {
        if (!m->geom_contype[g2] && !m->geom_conaffinity[g2]) continue;
        if (geom_filter_skip(m, g1, g2)) continue;
        if (is_convex_pair(m, g1, g2) != pass) continue;
        double r1 = m->geom_rbound[g1], r2 = m->geom_rbound[g2];
        double margin = fmax(m->geom_margin[g1], m->geom_margin[g2]);
        if (r1 > 0 && r2 > 0) {
          const double *a = d->geom_xpos + 3 * g1, *b = d->geom_xpos + 3 * g2;
          double v[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
          if (sqrt(dot3(v, v)) > r1 + r2 + margin) continue;
        }
        int room = ORC_MAXCON - d->ncon;
        if (room <= 0) { d->warn |= ORC_WARN_CONTACTFULL; return d->ncon; }
        d->ncon += orc_collide_pair(m, d, g1, g2, d->contact + d->ncon, room);
      }
    }
  return d->ncon;
}
