/* convex.c — convex narrowphase for mesh pairs (box-mesh, sphere-mesh, mesh-mesh): MuJoCo 2.3.3
 * mjc_Convex (engine_collision_convex.c) = libccd ccdMPRPenetration (Minkowski Portal
 * Refinement, libccd 2.x src/mpr.c, as vendored by MuJoCo) over geom support functions.
 * TEST INFRASTRUCTURE ONLY (see oracle.c).
 *
 * Restated from the published algorithm (third-party code absent here):
 *   discover a portal (center ray + 3 support points) -> refine until it contains the origin ->
 *   refine towards the surface until the support gain is within mpr_tolerance (1e-6, at most
 *   mpr_iterations = 50) -> depth = distance from the origin to the portal triangle, direction =
 *   its witness, position = barycentric mix of the two objects' support points (midpoint).
 *   Contact: dist = margin - depth, normal = direction (geom1 -> geom2), one contact per pair.
 * Supports (mjccd_support): box = centre + R sign(R^T d) size, sphere = centre + r d, mesh = the
 * hull vertex maximising d, each inflated by margin/2 along d; ties are resolved with a 1e-9 band
 * (first vertex within it of the maximum, + box corner for |d_k| < 1e-12) so that flat faces
 * facing each other — a finger hull on a shelf board — do not flip the portal with rounding.
 * mjc_MPRIteration: an MPR contact whose normal is undefined (zero) is dropped; mjc_fixNormal
 * replaces the normal by the analytic one for smooth geoms (here: the sphere, the only smooth
 * type in a convex pair of this scene).
 * multiccd (shelf_pnp.xml:5 enables it; mjENBL_MULTICCD in mjc_Convex): after the first contact,
 * MPR is re-run four times with the two geoms rotated in opposite senses ABOUT THE FIRST CONTACT'S
 * POSITION (mjc_rotateFrame) by +-perturbation_angle (1e-3 rad) about the two tangent axes of the
 * first contact's frame (mju_makeFrame of its normal): (t1, -a), (t1, +a), (t2, -a), (t2, +a),
 * geom 1 by q and geom 2 by q^-1.  A contact found this way is appended when its position is
 * farther than relative_tolerance (1e-3) x min(rbound1, rbound2) from every contact the pair
 * already has (up to 5 per pair).  Pairs with a smooth geom (the sphere) make no fan.
 * UNVERIFIED ASSUMPTIONS (MuJoCo 2.3.3's engine_collision_convex.c is not present here; the two
 * choices below follow two independent recollections of it -- round 3 rotated about the geoms'
 * own centres and fanned sphere pairs too): the rotation centre (the first contact point), the
 * sphere exclusion, the constants and the trial order.  Parity unpinned, DESIGN.md section 2.
 * Pairs whose oriented bounding boxes are disjoint cannot touch; they skip MPR (result-neutral).
 */
#include <float.h>
#include <math.h>
#include <string.h>

#include "physics.h"
#include "spatial.h"

typedef const pnp_model_desc Mdl;

enum { C_SPHERE = 2, C_BOX = 6, C_MESH = 7 };
#define MPR_TOL 1e-6
#define MPR_ITERS 50
#define CCD_EPS DBL_EPSILON
#define SUPP_TIE 1e-9   /* support ties (m): flat faces of both shapes, see support() */

typedef struct {
  Mdl* m;
  int type, mesh;
  double pos[3], R[9], size[3], margin;
} shape;

typedef struct {
  double v[3], v1[3], v2[3];   /* Minkowski point v = v1 - v2 and the supports it came from */
} svert;

/* MPR work counters (diagnostics: tools/mpr_census.py, single-threaded use only): runs, support
 * pairs (mk_support calls), discover / refine / penetration loop trips, runs that hit the
 * penetration loop's cap, and the largest support count of one run */
static _Thread_local long long g_mpr[8];   /* per thread: the pthread baseline never reads them */
void orc_mpr_stats(long long* out, int reset) {
  for (int i = 0; i < 8; i++) {
    out[i] = g_mpr[i];
    if (reset) g_mpr[i] = 0;
  }
}
static _Thread_local long long g_mpr_run_supports;

static int is_zero(double x) { return fabs(x) < CCD_EPS; }
static int ccd_eq(double a, double b) {
  double ab = fabs(a - b);
  if (ab < CCD_EPS) return 1;
  a = fabs(a);
  b = fabs(b);
  return b > a ? ab < CCD_EPS * b : ab < CCD_EPS * a;
}
static double d3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void c3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void sub3(double* r, const double* a, const double* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
/* ccdVec3Normalize: scale by the reciprocal of the length (one division, as libccd does) */
static void normalize(double* v) {
  const double k = 1.0 / sqrt(d3(v, v));
  v[0] *= k; v[1] *= k; v[2] *= k;
}

/* mjccd_support: support point of one geom along world direction d (unit) */
static void support(const shape* s, const double* d, double* out) {
  double ld[3];   /* d in the geom frame: R^T d */
  for (int k = 0; k < 3; k++) ld[k] = s->R[k] * d[0] + s->R[3 + k] * d[1] + s->R[6 + k] * d[2];
  double lp[3] = {0, 0, 0};
  if (s->type == C_SPHERE) {
    for (int k = 0; k < 3; k++) lp[k] = ld[k] * s->size[0];
  } else if (s->type == C_BOX) {
    /* the + corner when the direction is (within 1e-12) perpendicular to an axis: a face
       exactly facing the other shape must not flip with rounding */
    for (int k = 0; k < 3; k++) lp[k] = ld[k] >= -1e-12 ? s->size[k] : -s->size[k];
  } else {
    /* first vertex within SUPP_TIE of the maximum (flat hull faces tie exactly) */
    const double* V = s->m->mesh_vert + 3 * s->m->mesh_vertadr[s->mesh];
    int n = s->m->mesh_vertnum[s->mesh], best = 0;
    double bd = -DBL_MAX;
    for (int i = 0; i < n; i++) {
      double v = V[3 * i] * ld[0] + V[3 * i + 1] * ld[1] + V[3 * i + 2] * ld[2];
      if (v > bd) bd = v;
    }
    for (int i = 0; i < n; i++) {
      double v = V[3 * i] * ld[0] + V[3 * i + 1] * ld[1] + V[3 * i + 2] * ld[2];
      if (v >= bd - SUPP_TIE) { best = i; break; }
    }
    lp[0] = V[3 * best]; lp[1] = V[3 * best + 1]; lp[2] = V[3 * best + 2];
  }
  for (int k = 0; k < 3; k++)
    out[k] = s->pos[k] + s->R[3 * k] * lp[0] + s->R[3 * k + 1] * lp[1] + s->R[3 * k + 2] * lp[2] + 0.5 * s->margin * d[k];
}

/* __ccdSupport: v1 = supp1(d), v2 = supp2(-d), v = v1 - v2 */
static void mk_support(const shape* a, const shape* b, const double* d, svert* v) {
  double nd[3] = {-d[0], -d[1], -d[2]};
  g_mpr[1]++;
  g_mpr_run_supports++;
  support(a, d, v->v1);
  support(b, nd, v->v2);
  sub3(v->v, v->v1, v->v2);
}

static void portal_dir(const svert* p, double* dir) {
  double a[3], b[3];
  sub3(a, p[2].v, p[1].v);
  sub3(b, p[3].v, p[1].v);
  c3(dir, a, b);
  normalize(dir);
}
static int encapsules_origin(const svert* p, const double* dir) {
  double dot = d3(dir, p[1].v);
  return is_zero(dot) || dot > 0;
}
static int reach_tolerance(const svert* p, const svert* v4, const double* dir) {
  double dv1 = d3(p[1].v, dir), dv2 = d3(p[2].v, dir), dv3 = d3(p[3].v, dir), dv4 = d3(v4->v, dir);
  double t1 = dv4 - dv1, t2 = dv4 - dv2, t3 = dv4 - dv3;
  t1 = t1 < t2 ? t1 : t2;
  t1 = t1 < t3 ? t1 : t3;
  return ccd_eq(t1, MPR_TOL) || t1 < MPR_TOL;
}
static int can_encapsule(const svert* v4, const double* dir) {
  double dot = d3(v4->v, dir);
  return is_zero(dot) || dot > 0;
}
static void expand_portal(svert* p, const svert* v4) {
  double v4v0[3];
  c3(v4v0, v4->v, p[0].v);
  if (d3(p[1].v, v4v0) > 0) {
    if (d3(p[2].v, v4v0) > 0) p[1] = *v4;
    else p[3] = *v4;
  } else {
    if (d3(p[3].v, v4v0) > 0) p[2] = *v4;
    else p[1] = *v4;
  }
}

/* returns -1 no intersection, 0 portal found, 1 origin on v1, 2 origin on segment v0-v1 */
static int discover_portal(const shape* a, const shape* b, svert* p) {
  double dir[3], va[3], vb[3], dot;
  memcpy(p[0].v1, a->pos, sizeof(p[0].v1));
  memcpy(p[0].v2, b->pos, sizeof(p[0].v2));
  sub3(p[0].v, p[0].v1, p[0].v2);
  if (p[0].v[0] == 0 && p[0].v[1] == 0 && p[0].v[2] == 0) p[0].v[0] += CCD_EPS * 10.0;
  dir[0] = -p[0].v[0]; dir[1] = -p[0].v[1]; dir[2] = -p[0].v[2];
  normalize(dir);
  mk_support(a, b, dir, &p[1]);
  dot = d3(p[1].v, dir);
  if (is_zero(dot) || dot < 0) return -1;
  c3(dir, p[0].v, p[1].v);
  if (is_zero(d3(dir, dir))) {
    if (p[1].v[0] == 0 && p[1].v[1] == 0 && p[1].v[2] == 0) return 1;
    return 2;
  }
  normalize(dir);
  mk_support(a, b, dir, &p[2]);
  dot = d3(p[2].v, dir);
  if (is_zero(dot) || dot < 0) return -1;
  sub3(va, p[1].v, p[0].v);
  sub3(vb, p[2].v, p[0].v);
  c3(dir, va, vb);
  normalize(dir);
  if (d3(dir, p[0].v) > 0) {
    svert t = p[1];
    p[1] = p[2];
    p[2] = t;
    dir[0] = -dir[0]; dir[1] = -dir[1]; dir[2] = -dir[2];
  }
  for (int guard = 0; guard < 1000; guard++) {
    g_mpr[2]++;
    mk_support(a, b, dir, &p[3]);
    dot = d3(p[3].v, dir);
    if (is_zero(dot) || dot < 0) return -1;
    int cont = 0;
    c3(va, p[1].v, p[3].v);
    dot = d3(va, p[0].v);
    if (dot < 0 && !is_zero(dot)) {
      p[2] = p[3];
      cont = 1;
    }
    if (!cont) {
      c3(va, p[3].v, p[2].v);
      dot = d3(va, p[0].v);
      if (dot < 0 && !is_zero(dot)) {
        p[1] = p[3];
        cont = 1;
      }
    }
    if (!cont) return 0;
    sub3(va, p[1].v, p[0].v);
    sub3(vb, p[2].v, p[0].v);
    c3(dir, va, vb);
    normalize(dir);
  }
  return -1;
}

static int refine_portal(const shape* a, const shape* b, svert* p) {
  double dir[3];
  svert v4;
  for (int guard = 0; guard < 1000; guard++) {
    g_mpr[3]++;
    portal_dir(p, dir);
    if (encapsules_origin(p, dir)) return 0;
    mk_support(a, b, dir, &v4);
    if (!can_encapsule(&v4, dir) || reach_tolerance(p, &v4, dir)) return -1;
    expand_portal(p, &v4);
  }
  return -1;
}

/* squared distance from P to segment x0-b and its witness */
static double point_segment_dist2(const double* P, const double* x0, const double* b, double* w) {
  double d[3], a[3], t;
  sub3(d, b, x0);
  sub3(a, x0, P);
  t = -d3(a, d) / d3(d, d);
  if (t < 0 || is_zero(t)) {
    memcpy(w, x0, 3 * sizeof(double));
  } else if (t > 1 || ccd_eq(t, 1)) {
    memcpy(w, b, 3 * sizeof(double));
  } else {
    for (int k = 0; k < 3; k++) w[k] = d[k] * t + x0[k];
  }
  double e[3];
  sub3(e, w, P);
  return d3(e, e);
}

/* squared distance from P to triangle (x0, B, C) and its witness (ccdVec3PointTriDist2) */
static double point_tri_dist2(const double* P, const double* x0, const double* B, const double* C, double* w) {
  double d1[3], d2[3], a[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  sub3(a, x0, P);
  double u = d3(a, a), v = d3(d1, d1), ww = d3(d2, d2), p = d3(a, d1), q = d3(a, d2), r = d3(d1, d2);
  (void)u;
  double det = ww * v - r * r, s, t;
  if (is_zero(det)) {
    s = t = -1.0;
  } else {
    s = (q * r - ww * p) / det;
    t = (-s * r - q) / ww;
  }
  if ((is_zero(s) || s > 0) && (ccd_eq(s, 1) || s < 1) && (is_zero(t) || t > 0) && (ccd_eq(t, 1) || t < 1) &&
      (ccd_eq(t + s, 1) || t + s < 1)) {
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    double e[3];
    sub3(e, w, P);
    return d3(e, e);
  }
  double w2[3];
  double dist = point_segment_dist2(P, x0, B, w);
  double dist2 = point_segment_dist2(P, x0, C, w2);
  if (dist2 < dist) { dist = dist2; memcpy(w, w2, sizeof(w2)); }
  dist2 = point_segment_dist2(P, B, C, w2);
  if (dist2 < dist) { dist = dist2; memcpy(w, w2, sizeof(w2)); }
  return dist;
}

static void find_pos(const svert* p, double* pos) {
  double dir[3], vec[3], b[4], sum;
  portal_dir(p, dir);
  c3(vec, p[1].v, p[2].v);
  b[0] = d3(vec, p[3].v);
  c3(vec, p[3].v, p[2].v);
  b[1] = d3(vec, p[0].v);
  c3(vec, p[0].v, p[1].v);
  b[2] = d3(vec, p[3].v);
  c3(vec, p[2].v, p[1].v);
  b[3] = d3(vec, p[0].v);
  sum = b[0] + b[1] + b[2] + b[3];
  if (is_zero(sum) || sum < 0) {
    b[0] = 0;
    c3(vec, p[2].v, p[3].v);
    b[1] = d3(vec, dir);
    c3(vec, p[3].v, p[1].v);
    b[2] = d3(vec, dir);
    c3(vec, p[1].v, p[2].v);
    b[3] = d3(vec, dir);
    sum = b[1] + b[2] + b[3];
  }
  double inv = 1.0 / sum, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) {
      p1[k] += b[i] * p[i].v1[k];
      p2[k] += b[i] * p[i].v2[k];
    }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] * inv + p2[k] * inv);
}

/* ccdMPRPenetration: 0 and (depth, dir, pos) on intersection, -1 otherwise */
static int mpr_penetration_(const shape* a, const shape* b, double* depth, double* dir, double* pos);
static int mpr_penetration(const shape* a, const shape* b, double* depth, double* dir, double* pos) {
  g_mpr[0]++;
  g_mpr_run_supports = 0;
  const int r = mpr_penetration_(a, b, depth, dir, pos);
  if (g_mpr_run_supports > g_mpr[6]) g_mpr[6] = g_mpr_run_supports;
  return r;
}
static int mpr_penetration_(const shape* a, const shape* b, double* depth, double* dir, double* pos) {
  svert p[4];
  int res = discover_portal(a, b, p);
  if (res < 0) return -1;
  if (res == 1) {            /* touching on v1 */
    *depth = 0;
    dir[0] = dir[1] = dir[2] = 0;
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].v1[k] + p[1].v2[k]);
    return 0;
  }
  if (res == 2) {            /* origin on the segment v0-v1 */
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].v1[k] + p[1].v2[k]);
    memcpy(dir, p[1].v, 3 * sizeof(double));
    *depth = sqrt(d3(dir, dir));
    normalize(dir);
    return 0;
  }
  if (refine_portal(a, b, p) < 0) return -1;
  svert v4;
  double d[3];
  for (int it = 0;; it++) {
    g_mpr[4]++;
    portal_dir(p, d);
    mk_support(a, b, d, &v4);
    if (it > MPR_ITERS) g_mpr[5]++;
    if (reach_tolerance(p, &v4, d) || it > MPR_ITERS) {
      static const double O[3] = {0, 0, 0};
      *depth = sqrt(point_tri_dist2(O, p[1].v, p[2].v, p[3].v, dir));
      if (is_zero(*depth)) dir[0] = dir[1] = dir[2] = 0;
      else normalize(dir);
      find_pos(p, pos);
      return 0;
    }
    expand_portal(p, &v4);
  }
}

/* geom-frame bounding box: centre offset c and half extents h */
static void local_box(Mdl* m, int g, double* c, double* h) {
  int t = m->geom_type[g];
  c[0] = c[1] = c[2] = 0;
  if (t == C_SPHERE) { h[0] = h[1] = h[2] = m->geom_size[3 * g]; return; }
  if (t == C_BOX) { for (int k = 0; k < 3; k++) h[k] = m->geom_size[3 * g + k]; return; }
  int mesh = m->geom_dataid[g];
  const double* V = m->mesh_vert + 3 * m->mesh_vertadr[mesh];
  double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
  for (int i = 0; i < m->mesh_vertnum[mesh]; i++)
    for (int k = 0; k < 3; k++) {
      if (V[3 * i + k] < lo[k]) lo[k] = V[3 * i + k];
      if (V[3 * i + k] > hi[k]) hi[k] = V[3 * i + k];
    }
  for (int k = 0; k < 3; k++) { c[k] = 0.5 * (lo[k] + hi[k]); h[k] = 0.5 * (hi[k] - lo[k]); }
}

/* separating-axis test of two oriented boxes (15 axes), boxes inflated by margin */
static int obb_disjoint(const double* p1, const double* R1, const double* h1, const double* p2, const double* R2,
                        const double* h2, double margin) {
  double A[3][3], B[3][3], T[3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = R1[3 * k + i]; B[i][k] = R2[3 * k + i]; }
  sub3(T, p2, p1);
  double axes[15][3];
  int na = 0;
  for (int i = 0; i < 3; i++) memcpy(axes[na++], A[i], sizeof(A[i]));
  for (int i = 0; i < 3; i++) memcpy(axes[na++], B[i], sizeof(B[i]));
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) c3(axes[na++], A[i], B[j]);
  for (int a = 0; a < na; a++) {
    const double* L = axes[a];
    double len2 = d3(L, L);
    if (len2 < 1e-12) continue;
    double ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) { ra += h1[k] * fabs(d3(A[k], L)); rb += h2[k] * fabs(d3(B[k], L)); }
    if (fabs(d3(T, L)) > ra + rb + margin * sqrt(len2)) return 1;
  }
  return 0;
}

/* mjc_MPRIteration: one MPR run; 1 and the contact (normal fixed, mjc_fixNormal) on contact */
static int mpr_contact(const shape* s, double margin, orc_contact* c) {
  double depth, dir[3], pos[3];
  if (mpr_penetration(&s[0], &s[1], &depth, dir, pos) != 0) return 0;
  if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) return 0;   /* normal undefined */
  c->dist = margin - depth;
  memcpy(c->pos, pos, sizeof(pos));
  memset(c->frame, 0, sizeof(c->frame));
  memcpy(c->frame, dir, sizeof(dir));
  /* mjc_fixNormal: the sphere's normal at the contact point (from its centre, unperturbed
     frame); sphere is geom 1 of its pairs (lower type), its normal points to geom 2.  Both
     smooth would average; a second smooth geom does not occur (g2 is a mesh). */
  if (s[0].type == C_SPHERE) {
    double n[3];
    sub3(n, c->pos, s[0].pos);
    double len = sqrt(d3(n, n));
    if (len < 1e-15) { n[0] = 1; n[1] = n[2] = 0; }
    else { n[0] /= len; n[1] /= len; n[2] /= len; }
    memcpy(c->frame, n, sizeof(n));
  }
  return 1;
}

static int mpr_fan(Mdl* m, shape* s, int g1, int g2, double margin, orc_contact* out, int cap);

int orc_convex_collide(Mdl* m, const orc_data* d, int g1, int g2, double margin, orc_contact* out, int cap) {
  if (cap < 1) return 0;
  shape s[2];
  int gs[2] = {g1, g2};
  double bc[2][3], bh[2][3], bp[2][3];
  for (int i = 0; i < 2; i++) {
    int g = gs[i];
    s[i].m = m;
    s[i].type = m->geom_type[g];
    s[i].mesh = m->geom_dataid[g];
    s[i].margin = margin;
    memcpy(s[i].pos, d->geom_xpos + 3 * g, sizeof(s[i].pos));
    memcpy(s[i].R, d->geom_xmat + 9 * g, sizeof(s[i].R));
    for (int k = 0; k < 3; k++) s[i].size[k] = m->geom_size[3 * g + k];
    local_box(m, g, bc[i], bh[i]);
    for (int k = 0; k < 3; k++)
      bp[i][k] = s[i].pos[k] + s[i].R[3 * k] * bc[i][0] + s[i].R[3 * k + 1] * bc[i][1] + s[i].R[3 * k + 2] * bc[i][2];
  }
  if (obb_disjoint(bp[0], s[0].R, bh[0], bp[1], s[1].R, bh[1], margin)) return 0;
  /* MPR runs with the origin at geom 1's centre (support points of centimetre magnitude instead of
     world coordinates ~1 m: the fp32 kernel's Minkowski differences keep 20x more bits; a
     translation of both shapes leaves the algorithm's result unchanged) */
  const double o[3] = {s[0].pos[0], s[0].pos[1], s[0].pos[2]};
  for (int i = 0; i < 2; i++) sub3(s[i].pos, s[i].pos, o);
  int n = mpr_fan(m, s, g1, g2, margin, out, cap);
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) out[i].pos[k] += o[k];
  return n;
}

/* mjc_Convex after the pre-test: MPR, then multiccd's perturbed runs */
static int mpr_fan(Mdl* m, shape* s, int g1, int g2, double margin, orc_contact* out, int cap) {
  if (!mpr_contact(s, margin, &out[0])) return 0;
  int n = 1;
  if (!m->multiccd) return n;
  /* smooth geoms (the sphere) make no fan: assumed from MuJoCo's mjc_Convex (unverified, see the
     header) -- rotating a sphere about the contact point only slides it along its own surface */
  if (s[0].type == C_SPHERE || s[1].type == C_SPHERE) return n;
  /* multiccd: perturbed runs about the first contact's tangent axes */
  const double relative_tolerance = 1e-3, perturbation_angle = 1e-3;
  double frame[9];
  memcpy(frame, out[0].frame, sizeof(frame));
  frame[3] = frame[4] = frame[5] = 0;
  sp_makeframe(frame);
  double r1 = m->geom_rbound[g1], r2 = m->geom_rbound[g2];
  const double tol = relative_tolerance * (r1 < r2 ? r1 : r2);
  const double R0[2][9] = {
      {s[0].R[0], s[0].R[1], s[0].R[2], s[0].R[3], s[0].R[4], s[0].R[5], s[0].R[6], s[0].R[7], s[0].R[8]},
      {s[1].R[0], s[1].R[1], s[1].R[2], s[1].R[3], s[1].R[4], s[1].R[5], s[1].R[6], s[1].R[7], s[1].R[8]}};
  const double P0[2][3] = {{s[0].pos[0], s[0].pos[1], s[0].pos[2]}, {s[1].pos[0], s[1].pos[1], s[1].pos[2]}};
  const double* org = out[0].pos;   /* the rotations' centre: the first contact's position */
  for (int ax = 0; ax < 2; ax++)
    for (int sg = 0; sg < 2; sg++) {
      const double ang = sg ? perturbation_angle : -perturbation_angle;
      double q[4], qi[4], Rq[9], Rqi[9];
      sp_axisangle2quat(q, frame + 3 + 3 * ax, ang);
      sp_negquat(qi, q);
      sp_quat2mat(Rq, q);
      sp_quat2mat(Rqi, qi);
      /* (mjc_rotateFrame) geom 1 rotated by q, geom 2 by q^-1, both about the first contact */
      const double* Rs[2] = {Rq, Rqi};
      for (int i = 0; i < 2; i++) {
        double rel[3], rot[3];
        mulmat3(s[i].R, Rs[i], R0[i]);
        sub3(rel, P0[i], org);
        for (int k = 0; k < 3; k++) rot[k] = Rs[i][3 * k] * rel[0] + Rs[i][3 * k + 1] * rel[1] + Rs[i][3 * k + 2] * rel[2];
        for (int k = 0; k < 3; k++) s[i].pos[k] = org[k] + rot[k];
      }
      orc_contact c;
      if (!mpr_contact(s, margin, &c)) continue;
      int distinct = 1;
      for (int i = 0; i < n; i++) {
        double e[3];
        sub3(e, c.pos, out[i].pos);
        if (sqrt(d3(e, e)) <= tol) { distinct = 0; break; }
      }
      if (distinct && n < cap) out[n++] = c;
    }
  return n;
}

/* test probe: MPR on any (sphere | box | mesh) geom pair of a forward'ed orc_data, no OBB
 * pre-test; returns 1 and (dist, pos, normal) on contact */
int orc_convex_probe(Mdl* m, const orc_data* d, int g1, int g2, double* dist, double* pos, double* normal) {
  shape s[2];
  int gs[2] = {g1, g2};
  for (int i = 0; i < 2; i++) {
    int g = gs[i];
    s[i].m = m;
    s[i].type = m->geom_type[g];
    s[i].mesh = m->geom_dataid[g];
    s[i].margin = 0;
    memcpy(s[i].pos, d->geom_xpos + 3 * g, sizeof(s[i].pos));
    memcpy(s[i].R, d->geom_xmat + 9 * g, sizeof(s[i].R));
    for (int k = 0; k < 3; k++) s[i].size[k] = m->geom_size[3 * g + k];
  }
  double depth;
  if (mpr_penetration(&s[0], &s[1], &depth, normal, pos) != 0) return 0;
  *dist = -depth;
  return 1;
}
