// collide_dev.h — narrowphase colliders of the step kernel (included by step.hip).
// Same algorithms, same contact conventions as oracle/collision.c (normal from geom1 to geom2,
// contact point midway between the surfaces, MuJoCo mj_contactParam mixing):
//   plane-sphere, plane-box (corners below the plane, <= 4), plane-mesh (<= 4 deepest hull
//   vertices), sphere-sphere, sphere-box, box-box (SAT over 15 axes + reference/incident face
//   clipping, edge-edge), and (sphere | box | mesh) x mesh by MPR (oracle/convex.c).
// One lane runs one candidate pair; results stay in the lane's registers/scratch until the
// wave-wide scan places them.
#pragma once

// Colliders emit contacts into a sink that writes straight into the env's LDS contact list and
// counts; with cap = 0 it only counts (phase 1 of the wave-wide ordered placement).  One sink
// type = one copy of every collider in the kernel (instruction-cache footprint), and no
// per-lane contact arrays, so nothing spills to scratch.
template <typename T>
struct LdsSink {
  Con<T>* base;
  int cap, n = 0;
  __device__ __forceinline__ void emit(T dist, const T pos[3], const T nrm[3]) {
    if (n < cap) {
      Con<T>& c = base[n];
      c.dist = dist;
      for (int k = 0; k < 3; k++) c.pos[k] = pos[k];
      for (int k = 0; k < 9; k++) c.frame[k] = 0;
      c.frame[0] = nrm[0]; c.frame[1] = nrm[1]; c.frame[2] = nrm[2];
    }
    n++;
  }
};

// staging sink (single-pass narrowphase): a wave-wide LDS slot counter; each contact records its
// producing lane and its number within the pair so it can be placed in order afterwards
template <typename T>
struct StageSink {
  int* counter;
  T (*val)[7];
  unsigned short* key;
  int lane, n = 0;
  __device__ __forceinline__ void emit(T dist, const T pos[3], const T nrm[3]) {
    const int slot = atomicAdd(counter, 1);
    if (slot < 64 && n < 16) {
      val[slot][0] = dist;
      for (int k = 0; k < 3; k++) { val[slot][1 + k] = pos[k]; val[slot][4 + k] = nrm[k]; }
      key[slot] = (unsigned short)(lane * 16 + n);
    }
    n++;
  }
};

template <typename T, class S>
__device__ void c_plane_sphere(const T* p1, const T* R1, const T* p2, T r, T margin, S& out) {
  const T n[3] = {R1[2], R1[5], R1[8]}, v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const T dist = t_dot3(v, n) - r;
  if (dist > margin) return;
  T pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p2[k] - n[k] * (r + dist * T(0.5));
  out.emit(dist, pos, n);
}

template <typename T, class S>
__device__ void c_plane_box(const T* p1, const T* R1, const T* p2, const T* R2, const T* s, T margin, S& out) {
  const T n[3] = {R1[2], R1[5], R1[8]}, v[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const T dist = t_dot3(v, n);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    const T cr[3] = {(i & 1) ? s[0] : -s[0], (i & 2) ? s[1] : -s[1], (i & 4) ? s[2] : -s[2]};
    T w[3];
    d_mulmatvec3(w, R2, cr);
    const T ld = t_dot3(n, w);
    if (dist + ld > margin || ld > 0) continue;
    const T dd = dist + ld;
    T pos[3];
    for (int k = 0; k < 3; k++) pos[k] = w[k] + p2[k] - n[k] * dd * T(0.5);
    out.emit(dd, pos, n);
    if (++cnt >= 4) return;
  }
}

template <typename T, class S>
__device__ void c_plane_mesh(const DevPhys<T>& /*image: phys<T>()*/, const T* p1, const T* R1, const T* p2, const T* R2, int mesh, T margin,
                             S& out) {
  const DevPhys<T>& m = phys<T>();
  const T n[3] = {R1[2], R1[5], R1[8]};
  const int a = m.mesh_vertadr[mesh], nv = m.mesh_vertnum[mesh];
  T best[4];
  int bi[4], cnt = 0;
  for (int i = 0; i < nv; i++) {
    T w[3];
    d_mulmatvec3(w, R2, m.mesh_vert[a + i]);
    const T dd = (w[0] + p2[0] - p1[0]) * n[0] + (w[1] + p2[1] - p1[1]) * n[1] + (w[2] + p2[2] - p1[2]) * n[2];
    if (dd > margin) continue;
    int pos = cnt < 4 ? cnt : 4;
    while (pos > 0 && best[pos - 1] > dd) pos--;
    if (pos >= 4) continue;
    for (int k = (cnt < 4 ? cnt : 3); k > pos; k--) { best[k] = best[k - 1]; bi[k] = bi[k - 1]; }
    best[pos] = dd;
    bi[pos] = i;
    if (cnt < 4) cnt++;
  }
  for (int k = 0; k < cnt; k++) {
    T w[3], pos[3];
    d_mulmatvec3(w, R2, m.mesh_vert[a + bi[k]]);
    for (int t = 0; t < 3; t++) pos[t] = w[t] + p2[t] - n[t] * best[k] * T(0.5);
    out.emit(best[k], pos, n);
  }
}

template <typename T, class S>
__device__ void c_sphere_sphere(const T* p1, T r1, const T* p2, T r2, T margin, S& out) {
  T n[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const T len = PM<T>::sqrt_(t_dot3(n, n));
  const T dist = len - r1 - r2;
  if (dist > margin) return;
  if (len < T(1e-15)) { n[0] = 1; n[1] = 0; n[2] = 0; }
  else { n[0] /= len; n[1] /= len; n[2] /= len; }
  T pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * (r1 + dist * T(0.5));
  out.emit(dist, pos, n);
}

template <typename T, class S>
__device__ void c_sphere_box(const T* p1, T r, const T* p2, const T* R2, const T* s, T margin, S& out) {
  const T v[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  T lc[3], cl[3], nl[3], n[3];
  t_mulmattvec3(lc, R2, v);
  bool inside = true;
  for (int k = 0; k < 3; k++) {
    cl[k] = fmin(fmax(lc[k], -s[k]), s[k]);
    if (cl[k] != lc[k]) inside = false;
  }
  T dist;
  if (!inside) {
    for (int k = 0; k < 3; k++) nl[k] = cl[k] - lc[k];
    const T dd = PM<T>::sqrt_(t_dot3(nl, nl));
    dist = dd - r;
    if (dist > margin) return;
    for (int k = 0; k < 3; k++) nl[k] /= dd;
  } else {
    int kk = 0;
    T pen = s[0] - fabs(lc[0]);
    for (int k = 1; k < 3; k++)
      if (s[k] - fabs(lc[k]) < pen) { pen = s[k] - fabs(lc[k]); kk = k; }
    nl[0] = nl[1] = nl[2] = 0;
    nl[kk] = lc[kk] >= 0 ? T(-1) : T(1);
    dist = -(pen + r);
  }
  d_mulmatvec3(n, R2, nl);
  T pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * (r + dist * T(0.5));
  out.emit(dist, pos, n);
}

// 1 um band of oracle/collision.c BB_TOL (identical boxes face to face: robust decisions)
#define C_BB_TOL 1e-6

// Liang-Barsky clip of the 2D segment p0 -> p1 to |x| <= A, |y| <= B (closed); false if empty
template <typename T>
__device__ __forceinline__ bool c_clip_seg(const T* p0, const T* p1, T A, T B, T& t0, T& t1) {
  const T dx = p1[0] - p0[0], dy = p1[1] - p0[1];
  const T pp[4] = {-dx, dx, -dy, dy}, qq[4] = {p0[0] + A, A - p0[0], p0[1] + B, B - p0[1]};
  T a = 0, b = 1;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (pp[k] == T(0)) {
      ok &= !(qq[k] < T(0));
    } else {
      const T r = qq[k] / pp[k];
      if (pp[k] < T(0)) a = r > a ? r : a;
      else b = r < b ? r : b;
    }
  }
  t0 = a;
  t1 = b;
  return ok && !(a > b);
}

// Reference face on box r (axis ia, outward normal nr), incident box i (oracle/collision.c
// box_face_contacts, same vertex order): clipped incident-edge points, then reference corners
// strictly inside the incident face.  Fully unrolled: every array index is a compile-time
// constant, so the polygon lives in VGPRs (no private-memory scratch).
// Positions relative to the reference box: dpi = pi - pr (formed once from the two centres), the
// reference face centre at nr * sr[ia]; only the emitted contact position goes back to world
// coordinates.  (In fp32, world coordinates ~1 m carry 1e-7 m rounding, which the contact
// stiffness turns into a 1e-5-relative error of the reference acceleration; the box-frame
// differences here are ~0.05 m.)
template <typename T, class S>
__device__ void c_box_face(const T* pr, const T* Rr, const T* sr, int ia, const T* nr, const T* dpi, const T* Ri,
                           const T* si, const T* nframe, T margin, S& out) {
  const int iu = (ia + 1) % 3, iv = (ia + 2) % 3;
  const T u[3] = {Rr[iu], Rr[3 + iu], Rr[6 + iu]}, v[3] = {Rr[iv], Rr[3 + iv], Rr[6 + iv]};
  T cref[3];   // reference face centre relative to pr
  for (int k = 0; k < 3; k++) cref[k] = nr[k] * sr[ia];
  int ja = 0;
  T best = -1;
  for (int j = 0; j < 3; j++) {
    const T a = fabs(Ri[j] * nr[0] + Ri[3 + j] * nr[1] + Ri[6 + j] * nr[2]);
    if (a > best) { best = a; ja = j; }
  }
  const int ju = ja == 0 ? 1 : ja == 1 ? 2 : 0, jv = ja == 0 ? 2 : ja == 1 ? 0 : 1;
  const T bj[3] = {Ri[ja], Ri[3 + ja], Ri[6 + ja]};
  const T sg = t_dot3(bj, nr) > 0 ? T(-1) : T(1);
  const T bu[3] = {Ri[ju], Ri[3 + ju], Ri[6 + ju]}, bv[3] = {Ri[jv], Ri[3 + jv], Ri[6 + jv]};
  const T hj = si[ja], hu = si[ju], hv = si[jv];
  const T su[4] = {1, -1, -1, 1}, sv[4] = {1, 1, -1, -1};
  T P[4][3];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    T w[3];
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = dpi[k] + sg * bj[k] * hj + su[q] * bu[k] * hu + sv[q] * bv[k] * hv - cref[k];
    P[q][0] = t_dot3(w, u); P[q][1] = t_dot3(w, v); P[q][2] = t_dot3(w, nr);
  }
  const T A = sr[iu] + T(C_BB_TOL), B = sr[iv] + T(C_BB_TOL);   // rectangle grown by the band
  int cnt = 0;
  auto emit = [&](T x, T y, T z) {
    if (cnt >= 8 || z > margin + T(C_BB_TOL)) return;
    T pos[3];
#pragma unroll
    for (int k = 0; k < 3; k++) pos[k] = pr[k] + (cref[k] + u[k] * x + v[k] * y + nr[k] * z * T(0.5));
    out.emit(z, pos, nframe);
    cnt++;
  };
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const T* p0 = P[e];
    const T* p1 = P[(e + 1) & 3];
    T t0, t1;
    if (!c_clip_seg(p0, p1, A, B, t0, t1)) continue;
    emit(p0[0] + t0 * (p1[0] - p0[0]), p0[1] + t0 * (p1[1] - p0[1]), p0[2] + t0 * (p1[2] - p0[2]));
    if (t1 < T(1)) emit(p0[0] + t1 * (p1[0] - p0[0]), p0[1] + t1 * (p1[1] - p0[1]), p0[2] + t1 * (p1[2] - p0[2]));
  }
  const T e1[3] = {P[1][0] - P[0][0], P[1][1] - P[0][1], P[1][2] - P[0][2]};
  const T e3[3] = {P[3][0] - P[0][0], P[3][1] - P[0][1], P[3][2] - P[0][2]};
  const T det = e1[0] * e3[1] - e1[1] * e3[0];
  if (fabs(det) > T(1e-12) * (fabs(e1[0]) + fabs(e1[1])) * (fabs(e3[0]) + fabs(e3[1]))) {
    const T ta = T(C_BB_TOL) / PM<T>::sqrt_(e1[0] * e1[0] + e1[1] * e1[1]);
    const T tb = T(C_BB_TOL) / PM<T>::sqrt_(e3[0] * e3[0] + e3[1] * e3[1]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const T cx = su[q] * sr[iu] - P[0][0], cy = sv[q] * sr[iv] - P[0][1];
      const T al = (cx * e3[1] - cy * e3[0]) / det, be = (e1[0] * cy - e1[1] * cx) / det;
      if (al > ta && al < 1 - ta && be > tb && be < 1 - tb)
        emit(su[q] * sr[iu], sv[q] * sr[iv], P[0][2] + al * e1[2] + be * e3[2]);
    }
  }
}

template <typename T, class S>
__device__ void c_box_box(const T* p1, const T* R1, const T* s1, const T* p2, const T* R2, const T* s2, const T* Tv,
                          T margin, S& out) {
  T A[3][3], Bm[3][3], AB[3][3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = R1[3 * k + i]; Bm[i][k] = R2[3 * k + i]; }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) AB[i][j] = t_dot3(A[i], Bm[j]);
  T best = T(-1e30), bestn[3] = {0, 0, 0};
  int btype = -1, bi = 0, bj = 0;
  for (int i = 0; i < 3; i++) {
    const T tl = t_dot3(Tv, A[i]);
    const T rb = s2[0] * fabs(AB[i][0]) + s2[1] * fabs(AB[i][1]) + s2[2] * fabs(AB[i][2]);
    const T sep = fabs(tl) - s1[i] - rb;
    if (sep > margin) return;
    if (sep > best) { best = sep; btype = 0; bi = i; for (int k = 0; k < 3; k++) bestn[k] = tl >= 0 ? A[i][k] : -A[i][k]; }
  }
  for (int j = 0; j < 3; j++) {
    const T tl = t_dot3(Tv, Bm[j]);
    const T ra = s1[0] * fabs(AB[0][j]) + s1[1] * fabs(AB[1][j]) + s1[2] * fabs(AB[2][j]);
    const T sep = fabs(tl) - ra - s2[j];
    if (sep > margin) return;
    if (sep > best + T(C_BB_TOL)) { best = sep; btype = 1; bj = j; for (int k = 0; k < 3; k++) bestn[k] = tl >= 0 ? Bm[j][k] : -Bm[j][k]; }
  }
  // edge axes A_i x B_j in closed form from the direction cosines AB and the centre offset in
  // A's frame (Tv . (A_i x B_j) = ta_i2 AB_i1j - ta_i1 AB_i2j, |A_k . L|, |B_k . L| likewise); the
  // winning axis vector is formed once below
  T tA[3];
  for (int i = 0; i < 3; i++) tA[i] = t_dot3(Tv, A[i]);
  T btl = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      // |A_i x B_j|^2 = AB_i1j^2 + AB_i2j^2 (A orthonormal): no cancellation for near-parallel
      // edges, unlike 1 - AB_ij^2 in fp32
      const T len = PM<T>::sqrt_(AB[i1][j] * AB[i1][j] + AB[i2][j] * AB[i2][j]);
      if (len < T(1e-6)) continue;
      const T inv = T(1) / len;
      const T tl = (tA[i2] * AB[i1][j] - tA[i1] * AB[i2][j]) * inv;
      const T ra = (s1[i1] * fabs(AB[i2][j]) + s1[i2] * fabs(AB[i1][j])) * inv;
      const T rb = (s2[j1] * fabs(AB[i][j2]) + s2[j2] * fabs(AB[i][j1])) * inv;
      const T sep = fabs(tl) - ra - rb;
      if (sep > margin) return;
      if (T(1.05) * sep > best + T(C_BB_TOL)) {   // (oracle/collision.c A3: faces win near-ties)
        best = sep; btype = 2; bi = i; bj = j; btl = tl;
      }
    }
  }
  // rows A[bi], Bm[bj] by selects: a runtime index into the register arrays would put A and Bm in
  // scratch (six 12-byte spills and reloads per lane and box pair, every sub-step)
  T ua[3], ub[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    ua[k] = bi == 0 ? A[0][k] : (bi == 1 ? A[1][k] : A[2][k]);
    ub[k] = bj == 0 ? Bm[0][k] : (bj == 1 ? Bm[1][k] : Bm[2][k]);
  }
  if (btype == 2) {
    T L[3];
    t_cross(L, ua, ub);
    const T len = PM<T>::sqrt_(t_dot3(L, L));
    for (int k = 0; k < 3; k++) bestn[k] = btl >= 0 ? L[k] / len : -L[k] / len;
  }
  if (btype == 0) { c_box_face(p1, R1, s1, bi, bestn, Tv, R2, s2, bestn, margin, out); return; }
  if (btype == 1) {
    const T nr[3] = {-bestn[0], -bestn[1], -bestn[2]};
    const T dp1[3] = {-Tv[0], -Tv[1], -Tv[2]};
    c_box_face(p2, R2, s2, bj, nr, dp1, R1, s1, bestn, margin, out);
    return;
  }
  // edge-edge: the closest points of the two edges, relative to p1
  T pa[3] = {0, 0, 0}, pb[3] = {Tv[0], Tv[1], Tv[2]};
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (t != bi) {
      const T sg = t_dot3(A[t], bestn) > 0 ? T(1) : T(-1);
      for (int k = 0; k < 3; k++) pa[k] += sg * s1[t] * A[t][k];
    }
    if (t != bj) {
      const T sg = t_dot3(Bm[t], bestn) > 0 ? T(-1) : T(1);
      for (int k = 0; k < 3; k++) pb[k] += sg * s2[t] * Bm[t][k];
    }
  }
  const T w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
  const T a = t_dot3(ua, ub), dd = t_dot3(ua, w), e = t_dot3(ub, w), den = 1 - a * a;
  T ta = 0, tb = 0;
  if (den > T(1e-12)) { ta = (a * e - dd) / den; tb = (e - a * dd) / den; }
  for (int k = 0; k < 3; k++) { pa[k] += ta * ua[k]; pb[k] += tb * ub[k]; }
  T pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + T(0.5) * (pa[k] + pb[k]);
  out.emit(best, pos, bestn);
}

// mju_makeFrame: complete the contact frame from its normal (colliders set the normal only)
// ---------------------------------------------------------------- convex pairs (MPR)
// oracle/convex.c restated on the device (MuJoCo 2.3.3 mjc_Convex = libccd ccdMPRPenetration):
// same control flow and constants; the portal lives in registers (every index below is a
// compile-time constant).  The arithmetic is fp64 in every build (CT), the fp32 product kernels
// included (round 4): where the penetration direction is not unique (a hull corner on a board,
// two faces multiccd tilts 2e-3 rad apart) MPR's path decides the normal, and fp32 rounding of the
// Minkowski differences, portal sign tests and support gains took the other branch on a third of
// the convex-contact fixture's envs.  Inputs (geom frames, hull vertices) stay the build's T and are
// widened exactly; the contact leaves rounded to T.  The compact tier runs the first MPR only (a
// contact with multiccd hands the sub-step over), in its own out-of-line stage.
//
// Wave-cooperative: the whole wave runs MPR on ONE pair (every lane holds the same portal, so
// all branches are uniform) and splits each mesh support map over its 64 lanes.  Lane l keeps
// hull vertices l, l+64, l+128 in registers for the whole MPR run (CGrp<64>::NW per lane; larger hulls
// stream the rest from global memory), a support is three dot products, a DPP max and a ballot
// for the first vertex inside the tie band -- instead of 2 x nvert dependent global loads on a
// single lane.
// Lane groups (round 6): G lanes run one MPR -- G = 64, the whole wave (the serial pass, the fp64
// builds), or G = 16, one DPP row: four independent MPR runs per wave (the fp32 full / wide
// builds' convex pass, step.hip convex_part).  Every lane of a group holds the same portal (the
// group's branches are uniform) and the support maps split over the group's lanes; a group keeps
// CGrp<G>::NW hull vertices per lane in registers (G = 64: 192 vertices, G = 16: 64) and streams the
// rest from global memory.  The arithmetic of each lane is the same for both widths: the same bits.
template <int G> struct CGrp;
template <> struct CGrp<64> { static constexpr int NW = 3; };
template <> struct CGrp<16> { static constexpr int NW = 4; };
template <> struct CGrp<8> { static constexpr int NW = 8; };
#ifndef PNP_MPR_CT
#define PNP_MPR_CT double   // (A/B builds only: PNP_DEFS=-DPNP_MPR_CT=float)
#endif
typedef PNP_MPR_CT CT;   // MPR arithmetic (every build)
template <typename T, int G = 64>
struct CShape {
  static constexpr int NW = CGrp<G>::NW;
  int type, mesh, vadr, nvert;
  CT pos[3], R[9], size[3], margin;
  T wv[NW][3];   // mesh: vertices (lane in the group) + G j (local frame, the image's precision)
};
struct SVert {
  CT v[3], v1[3], v2[3];
};
template <typename T> __device__ __forceinline__ T ccd_eps() { return PM<T>::eps(); }
template <typename T> __device__ __forceinline__ bool ccd_zero(T x) { return fabs(x) < ccd_eps<T>(); }
template <typename T>
__device__ __forceinline__ bool ccd_eq(T a, T b) {
  const T ab = fabs(a - b);
  if (ab < ccd_eps<T>()) return true;
  a = fabs(a);
  b = fabs(b);
  return b > a ? ab < ccd_eps<T>() * b : ab < ccd_eps<T>() * a;
}
template <typename T> __device__ __forceinline__ T cd3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T>
__device__ __forceinline__ void cc3(T* r, const T* a, const T* b) {
  const T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <typename T> __device__ __forceinline__ void cs3(T* r, const T* a, const T* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
template <typename T>
__device__ __forceinline__ void cnorm(T* v) {   // ccdVec3Normalize: by the reciprocal length
  const T k = T(1) / PM<T>::sqrt_(cd3(v, v));
  v[0] *= k; v[1] *= k; v[2] *= k;
}
// max over the wave (all 64 lanes active), wave-uniform result
template <typename T>
__device__ __forceinline__ T c_wave_max(T v) {
  v = fmax(v, dpp_f<0xB1>(v));
  v = fmax(v, dpp_f<0x4E>(v));
  v = fmax(v, dpp_f<0x141>(v));
  v = fmax(v, dpp_f<0x140>(v));
  return fmax(fmax(rdlane(v, 0), rdlane(v, 16)), fmax(rdlane(v, 32), rdlane(v, 48)));
}
// max over the lane group (all its lanes active), group-uniform result
template <int G, typename T>
__device__ __forceinline__ T c_grp_max(T v) {
  if constexpr (G == 64) {
    return c_wave_max(v);
  } else if constexpr (G == 16) {
    return rowmax16(v);
  } else {   // G == 8: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror
    static_assert(G == 8, "lane group width");
    v = fmax(v, dpp_f<0xB1>(v));
    v = fmax(v, dpp_f<0x4E>(v));
    return fmax(v, dpp_f<0x141>(v));
  }
}
template <typename T, int G>
__device__ void c_load_shape(const DevPhys<T>& /*image: phys<T>()*/, CShape<T, G>& sh) {
  const DevPhys<T>& m = phys<T>();
  const int l = threadIdx.x & (G - 1);
  sh.vadr = sh.type == 7 ? m.mesh_vertadr[sh.mesh] : 0;
  sh.nvert = sh.type == 7 ? m.mesh_vertnum[sh.mesh] : 0;
#pragma unroll
  for (int j = 0; j < CShape<T, G>::NW; j++) {
    const int i = G * j + l;
    for (int k = 0; k < 3; k++) sh.wv[j][k] = i < sh.nvert ? m.mesh_vert[sh.vadr + i][k] : T(0);
  }
}
// the lane group's bits of a wave ballot (G = 64: all of them)
template <int G>
__device__ __forceinline__ uint64_t c_grp_bits(uint64_t b) {
  if constexpr (G == 64) return b;
  else return (b >> ((threadIdx.x & 63) & ~(G - 1))) & ((1ull << G) - 1ull);
}
// first vertex within the tie band of the maximum (oracle/convex.c support), group-cooperative
template <typename T, int G>
__device__ int c_mesh_argmax(const DevPhys<T>& /*image: phys<T>()*/, const CShape<T, G>& s, const CT* ld) {
  const DevPhys<T>& m = phys<T>();
  constexpr int NW = CShape<T, G>::NW;
  const int l = threadIdx.x & (G - 1), n = s.nvert;
  CT dv[NW], bd = CT(-1e30);
#pragma unroll
  for (int j = 0; j < NW; j++) {
    dv[j] = G * j + l < n ? CT(s.wv[j][0]) * ld[0] + CT(s.wv[j][1]) * ld[1] + CT(s.wv[j][2]) * ld[2] : CT(-1e30);
    bd = fmax(bd, dv[j]);
  }
  for (int i = G * NW + l; i < n; i += G) {
    const T* V = m.mesh_vert[s.vadr + i];
    bd = fmax(bd, CT(V[0]) * ld[0] + CT(V[1]) * ld[1] + CT(V[2]) * ld[2]);
  }
  bd = c_grp_max<G>(bd);
  const CT lo = bd - CT(1e-9);
#pragma unroll
  for (int j = 0; j < NW; j++) {
    const uint64_t b = c_grp_bits<G>(__ballot(G * j + l < n && dv[j] >= lo));
    if (b) return G * j + __ffsll((unsigned long long)b) - 1;
  }
  for (int base = G * NW; base < n; base += G) {
    const int i = base + l;
    bool ok = false;
    if (i < n) {
      const T* V = m.mesh_vert[s.vadr + i];
      ok = CT(V[0]) * ld[0] + CT(V[1]) * ld[1] + CT(V[2]) * ld[2] >= lo;
    }
    const uint64_t b = c_grp_bits<G>(__ballot(ok));
    if (b) return base + __ffsll((unsigned long long)b) - 1;
  }
  return 0;
}
template <typename T, int G>
__device__ void c_support(const DevPhys<T>& /*image: phys<T>()*/, const CShape<T, G>& s, const CT* d, CT* out) {
  const DevPhys<T>& m = phys<T>();
  CT ld[3];
  for (int k = 0; k < 3; k++) ld[k] = s.R[k] * d[0] + s.R[3 + k] * d[1] + s.R[6 + k] * d[2];
  CT lp[3];
  if (s.type == 2) {
    for (int k = 0; k < 3; k++) lp[k] = ld[k] * s.size[0];
  } else if (s.type == 6) {
    for (int k = 0; k < 3; k++) lp[k] = ld[k] >= CT(-1e-12) ? s.size[k] : -s.size[k];
  } else {
    const T* V = m.mesh_vert[s.vadr + c_mesh_argmax(m, s, ld)];
    lp[0] = V[0]; lp[1] = V[1]; lp[2] = V[2];
  }
  for (int k = 0; k < 3; k++)
    out[k] = s.pos[k] + s.R[3 * k] * lp[0] + s.R[3 * k + 1] * lp[1] + s.R[3 * k + 2] * lp[2] + CT(0.5) * s.margin * d[k];
}
template <typename T, int G>
__device__ __forceinline__ void c_mksupport(const DevPhys<T>& /*image: phys<T>()*/, const CShape<T, G>& a, const CShape<T, G>& b, const CT* d, SVert& v) {
  const DevPhys<T>& m = phys<T>();
  const CT nd[3] = {-d[0], -d[1], -d[2]};
  c_support(m, a, d, v.v1);
  c_support(m, b, nd, v.v2);
  cs3(v.v, v.v1, v.v2);
}
// Portal vertices in registers (SVert) or, in the full / wide builds, with their two support points in
// a per-wave LDS slot (SVertL: v in registers; v1 / v2 are read only by the touching case and
// findPos): 48 fewer fp64 VGPRs live across MPR's portal loops.  Slot ids are wave-uniform; a new
// support takes the slot no portal vertex holds.  Every lane writes the same values.
struct SVertL {
  CT v[3];
  int id;
};
template <typename T, int G>
__device__ __forceinline__ void c_mks(const DevPhys<T>& m, const CShape<T, G>& a, const CShape<T, G>& b, const CT* d, SVert& v,
                                      double (*)[6], int) {
  c_mksupport(m, a, b, d, v);
}
template <typename T, int G>
__device__ __forceinline__ void c_mks(const DevPhys<T>& m, const CShape<T, G>& a, const CShape<T, G>& b, const CT* d, SVertL& v,
                                      double (*sv)[6], int id) {
  SVert t;
  c_mksupport(m, a, b, d, t);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    v.v[k] = t.v[k];
    sv[id][k] = t.v1[k];
    sv[id][3 + k] = t.v2[k];
  }
  v.id = id;
}
__device__ __forceinline__ CT c_sv1(const SVert& p, double (*)[6], int k) { return p.v1[k]; }
__device__ __forceinline__ CT c_sv2(const SVert& p, double (*)[6], int k) { return p.v2[k]; }
__device__ __forceinline__ CT c_sv1(const SVertL& p, double (*sv)[6], int k) { return CT(sv[p.id][k]); }
__device__ __forceinline__ CT c_sv2(const SVertL& p, double (*sv)[6], int k) { return CT(sv[p.id][3 + k]); }
__device__ __forceinline__ int c_svid(const SVert&) { return 0; }
__device__ __forceinline__ int c_svid(const SVertL& p) { return p.id; }
template <typename V>
__device__ __forceinline__ void c_portal_dir(const V& p1, const V& p2, const V& p3, CT* dir) {
  CT a[3], b[3];
  cs3(a, p2.v, p1.v);
  cs3(b, p3.v, p1.v);
  cc3(dir, a, b);
  cnorm(dir);
}
template <typename V>
__device__ __forceinline__ bool c_reach_tol(const V& p1, const V& p2, const V& p3, const V& v4,
                                            const CT* dir, CT tol) {
  const CT dv4 = cd3(v4.v, dir);
  CT t1 = dv4 - cd3(p1.v, dir), t2 = dv4 - cd3(p2.v, dir), t3 = dv4 - cd3(p3.v, dir);
  t1 = t1 < t2 ? t1 : t2;
  t1 = t1 < t3 ? t1 : t3;
  return ccd_eq(t1, tol) || t1 < tol;
}
template <typename V>
__device__ __forceinline__ void c_expand(const SVert& p0, V& p1, V& p2, V& p3, const V& v4) {
  CT v4v0[3];
  cc3(v4v0, v4.v, p0.v);
  if (cd3(p1.v, v4v0) > 0) {
    if (cd3(p2.v, v4v0) > 0) p1 = v4;
    else p3 = v4;
  } else {
    if (cd3(p3.v, v4v0) > 0) p2 = v4;
    else p1 = v4;
  }
}
template <typename T>
__device__ T c_seg_dist2(const T* P, const T* x0, const T* b, T* w) {
  T d[3], a[3];
  cs3(d, b, x0);
  cs3(a, x0, P);
  const T t = -cd3(a, d) / cd3(d, d);
  if (t < 0 || ccd_zero(t)) {
    w[0] = x0[0]; w[1] = x0[1]; w[2] = x0[2];
  } else if (t > 1 || ccd_eq(t, T(1))) {
    w[0] = b[0]; w[1] = b[1]; w[2] = b[2];
  } else {
    for (int k = 0; k < 3; k++) w[k] = d[k] * t + x0[k];
  }
  T e[3];
  cs3(e, w, P);
  return cd3(e, e);
}
template <typename T>
__device__ T c_tri_dist2(const T* P, const T* x0, const T* B, const T* C, T* w) {
  T d1[3], d2[3], a[3];
  cs3(d1, B, x0);
  cs3(d2, C, x0);
  cs3(a, x0, P);
  const T v = cd3(d1, d1), ww = cd3(d2, d2), p = cd3(a, d1), q = cd3(a, d2), r = cd3(d1, d2);
  const T det = ww * v - r * r;
  T s, t;
  if (ccd_zero(det)) {
    s = t = T(-1);
  } else {
    s = (q * r - ww * p) / det;
    t = (-s * r - q) / ww;
  }
  if ((ccd_zero(s) || s > 0) && (ccd_eq(s, T(1)) || s < 1) && (ccd_zero(t) || t > 0) && (ccd_eq(t, T(1)) || t < 1) &&
      (ccd_eq(t + s, T(1)) || t + s < 1)) {
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    T e[3];
    cs3(e, w, P);
    return cd3(e, e);
  }
  T w2[3];
  T dist = c_seg_dist2(P, x0, B, w);
  T dist2 = c_seg_dist2(P, x0, C, w2);
  if (dist2 < dist) { dist = dist2; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  dist2 = c_seg_dist2(P, B, C, w2);
  if (dist2 < dist) { dist = dist2; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  return dist;
}

// ccdMPRPenetration: true and (depth, dir, pos) on intersection
template <typename T, typename V = SVert, int G = 64>
__device__ bool c_mpr(const DevPhys<T>& /*image: phys<T>()*/, const CShape<T, G>& A, const CShape<T, G>& Bs, CT& depth, CT* dir, CT* pos,
                      double (*sv)[6] = nullptr) {
  const DevPhys<T>& m = phys<T>();
  const CT tol = CT(1e-6);   // mjOption mpr_tolerance
  SVert p0;
  V p1, p2, p3, v4;
  CT d[3], va[3], vb[3], dot;
  // ---- discover portal
  for (int k = 0; k < 3; k++) { p0.v1[k] = A.pos[k]; p0.v2[k] = Bs.pos[k]; }
  cs3(p0.v, p0.v1, p0.v2);
  if (p0.v[0] == 0 && p0.v[1] == 0 && p0.v[2] == 0) p0.v[0] += ccd_eps<CT>() * CT(10);
  d[0] = -p0.v[0]; d[1] = -p0.v[1]; d[2] = -p0.v[2];
  cnorm(d);
  c_mks(m, A, Bs, d, p1, sv, 0);
  dot = cd3(p1.v, d);
  if (ccd_zero(dot) || dot < 0) return false;
  cc3(d, p0.v, p1.v);
  if (ccd_zero(cd3(d, d))) {
    for (int k = 0; k < 3; k++) pos[k] = CT(0.5) * (c_sv1(p1, sv, k) + c_sv2(p1, sv, k));
    if (p1.v[0] == 0 && p1.v[1] == 0 && p1.v[2] == 0) {   // touching on v1
      depth = 0;
      dir[0] = dir[1] = dir[2] = 0;
      return true;
    }
    for (int k = 0; k < 3; k++) dir[k] = p1.v[k];          // origin on the segment v0-v1
    depth = PM<CT>::sqrt_(cd3(dir, dir));
    cnorm(dir);
    return true;
  }
  cnorm(d);
  c_mks(m, A, Bs, d, p2, sv, 1);
  dot = cd3(p2.v, d);
  if (ccd_zero(dot) || dot < 0) return false;
  cs3(va, p1.v, p0.v);
  cs3(vb, p2.v, p0.v);
  cc3(d, va, vb);
  cnorm(d);
  if (cd3(d, p0.v) > 0) {
    const V t = p1;
    p1 = p2;
    p2 = t;
    d[0] = -d[0]; d[1] = -d[1]; d[2] = -d[2];
  }
  bool found = false;
  for (int guard = 0; guard < 1000 && !found; guard++) {
    c_mks(m, A, Bs, d, p3, sv, 3 - c_svid(p1) - c_svid(p2));
    dot = cd3(p3.v, d);
    if (ccd_zero(dot) || dot < 0) return false;
    bool cont = false;
    cc3(va, p1.v, p3.v);
    dot = cd3(va, p0.v);
    if (dot < 0 && !ccd_zero(dot)) { p2 = p3; cont = true; }
    if (!cont) {
      cc3(va, p3.v, p2.v);
      dot = cd3(va, p0.v);
      if (dot < 0 && !ccd_zero(dot)) { p1 = p3; cont = true; }
    }
    if (!cont) {
      found = true;
    } else {
      cs3(va, p1.v, p0.v);
      cs3(vb, p2.v, p0.v);
      cc3(d, va, vb);
      cnorm(d);
    }
  }
  if (!found) return false;
  // ---- refine until the portal contains the origin
  bool inside = false;
  for (int guard = 0; guard < 1000 && !inside; guard++) {
    c_portal_dir(p1, p2, p3, d);
    dot = cd3(d, p1.v);
    if (ccd_zero(dot) || dot > 0) { inside = true; break; }
    c_mks(m, A, Bs, d, v4, sv, 6 - c_svid(p1) - c_svid(p2) - c_svid(p3));
    dot = cd3(v4.v, d);
    if (!(ccd_zero(dot) || dot > 0) || c_reach_tol(p1, p2, p3, v4, d, tol)) return false;
    c_expand(p0, p1, p2, p3, v4);
  }
  if (!inside) return false;
  // ---- penetration: refine towards the surface
  for (int it = 0;; it++) {
    c_portal_dir(p1, p2, p3, d);
    c_mks(m, A, Bs, d, v4, sv, 6 - c_svid(p1) - c_svid(p2) - c_svid(p3));
    if (c_reach_tol(p1, p2, p3, v4, d, tol) || it > 50) {
      const CT O[3] = {0, 0, 0};
      depth = PM<CT>::sqrt_(c_tri_dist2(O, p1.v, p2.v, p3.v, dir));
      if (ccd_zero(depth)) dir[0] = dir[1] = dir[2] = 0;
      else cnorm(dir);
      // contact position: barycentric mix of the supports (findPos)
      CT vec[3], b0, b1, b2, b3;
      c_portal_dir(p1, p2, p3, d);
      cc3(vec, p1.v, p2.v); b0 = cd3(vec, p3.v);
      cc3(vec, p3.v, p2.v); b1 = cd3(vec, p0.v);
      cc3(vec, p0.v, p1.v); b2 = cd3(vec, p3.v);
      cc3(vec, p2.v, p1.v); b3 = cd3(vec, p0.v);
      CT sum = b0 + b1 + b2 + b3;
      if (ccd_zero(sum) || sum < 0) {
        b0 = 0;
        cc3(vec, p2.v, p3.v); b1 = cd3(vec, d);
        cc3(vec, p3.v, p1.v); b2 = cd3(vec, d);
        cc3(vec, p1.v, p2.v); b3 = cd3(vec, d);
        sum = b1 + b2 + b3;
      }
      const CT inv = CT(1) / sum;
      for (int k = 0; k < 3; k++) {
        const CT q1 = b0 * p0.v1[k] + b1 * c_sv1(p1, sv, k) + b2 * c_sv1(p2, sv, k) + b3 * c_sv1(p3, sv, k);
        const CT q2 = b0 * p0.v2[k] + b1 * c_sv2(p1, sv, k) + b2 * c_sv2(p2, sv, k) + b3 * c_sv2(p3, sv, k);
        pos[k] = CT(0.5) * (q1 * inv + q2 * inv);
      }
      return true;
    }
    c_expand(p0, p1, p2, p3, v4);
  }
}

// oriented-box separating-axis test (15 axes), boxes inflated by margin.  The classic form: the
// 9 direction cosines R = A^T B and the centre offset in both frames are formed once, then every
// axis is a few products of them -- all 15 evaluated branch-free (no per-axis early exit, so
// the wave's lanes stay converged).  Face axes: |t_i| > h1_i + sum_j h2_j |R_ij| + margin (and
// the same from B); edge axes A_i x B_j (skipped when parallel) compare the projections over
// |A_i x B_j| = sqrt(R_i1j^2 + R_i2j^2), the margin scaled by it as before.
template <typename T>
__device__ bool c_obb_disjoint(const T* p1, const T* R1, const T* h1, const T* p2, const T* R2, const T* h2, T margin) {
  T A[3][3], B[3][3], Tv[3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) { A[i][k] = R1[3 * k + i]; B[i][k] = R2[3 * k + i]; }
  cs3(Tv, p2, p1);
  T R[3][3], aR[3][3], ta[3], tb[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    ta[i] = cd3(Tv, A[i]);
    tb[i] = cd3(Tv, B[i]);
#pragma unroll
    for (int j = 0; j < 3; j++) { R[i][j] = cd3(A[i], B[j]); aR[i][j] = fabs(R[i][j]); }
  }
  bool sep = false;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const T rb = h2[0] * aR[i][0] + h2[1] * aR[i][1] + h2[2] * aR[i][2];
    sep |= fabs(ta[i]) > h1[i] + rb + margin;
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const T ra = h1[0] * aR[0][j] + h1[1] * aR[1][j] + h1[2] * aR[2][j];
    sep |= fabs(tb[j]) > ra + h2[j] + margin;
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      const T len2 = R[i1][j] * R[i1][j] + R[i2][j] * R[i2][j];   // |A_i x B_j|^2, cancellation-free
      const T d = fabs(ta[i2] * R[i1][j] - ta[i1] * R[i2][j]);
      const T ra = h1[i1] * aR[i2][j] + h1[i2] * aR[i1][j];
      const T rb = h2[j1] * aR[i][j2] + h2[j2] * aR[i][j1];
      sep |= len2 >= T(1e-12) && d > ra + rb + margin * PM<T>::sqrt_(len2 > T(0) ? len2 : T(0));
    }
  }
  return sep;
}

// convex pair: (sphere | box | mesh) x mesh (g1 has the lower type)
template <typename T>
__device__ __forceinline__ bool c_is_convex_pair(const DevPhys<T>& /*image: phys<T>()*/, int g1, int g2) {
  const DevPhys<T>& m = phys<T>();
  return m.geom_type[g2] == 7 && m.geom_type[g1] != 0;
}

// oriented bounding boxes of a convex pair disjoint (broadphase: such pairs cannot touch, MPR
// would find no contact)
template <typename T>
__device__ __forceinline__ bool c_convex_obb_disjoint(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2, T margin) {
  const DevPhys<T>& m = phys<T>();
  T bp[2][3];
  const int gs[2] = {g1, g2};
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int g = gs[i];
    const T* c = m.geom_aabb[g];
    const T* R = s.gmat[g];
    for (int k = 0; k < 3; k++) bp[i][k] = s.gpos[g][k] + R[3 * k] * c[0] + R[3 * k + 1] * c[1] + R[3 * k + 2] * c[2];
  }
  return c_obb_disjoint(bp[0], s.gmat[g1], m.geom_aabb[g1] + 3, bp[1], s.gmat[g2], m.geom_aabb[g2] + 3, margin);
}

// Compact tier's convex screen (instead of MPR): true only when the pair provably has no contact
// -- every hull vertex of mesh gm lies beyond one face plane of geom gb's bounding box (box:
// its own faces; mesh: its AABB, which holds its hull) by more than the margin plus 1e-5 m
// (fp32 rounding of the world-frame vertices is ~1e-7 m), or, for the sphere, beyond the plane at
// radius + margin + 1e-5 from its centre towards the hull's box centre.  The hull is the convex
// combination of its vertices, so it lies beyond that plane too: MPR (fp64, full tier) would find
// no contact.  Anything not proven separated hands the sub-step over, so the compact tier carries
// no MPR (its fp64 frame cost C3 2 %: scratch 704 -> 292 B per lane with it gone).
// Wave-cooperative: lane l takes vertices l, l + 64, l + 128 (hulls of up to 192 vertices; larger
// ones are never proven).
template <typename T>
__device__ bool c_hull_beyond(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int gm, int gb, T margin) {
  const DevPhys<T>& m = phys<T>();
  const int l = threadIdx.x & 63;
  const int mesh = m.geom_dataid[gm], n = m.mesh_vertnum[mesh], vadr = m.mesh_vertadr[mesh];
  if (n > 192) return false;
  const T* Rm = s.gmat[gm];
  const T* Rb = s.gmat[gb];
  const T* cb = m.geom_aabb[gb];
  const bool sph = m.geom_type[gb] == 2;
  T u[3] = {0, 0, 0};
  if (sph) {   // towards the hull's box centre
    const T* cm = m.geom_aabb[gm];
    T w[3], nn = 0;
    for (int k = 0; k < 3; k++) {
      w[k] = s.gpos[gm][k] + Rm[3 * k] * cm[0] + Rm[3 * k + 1] * cm[1] + Rm[3 * k + 2] * cm[2] - s.gpos[gb][k];
      nn += w[k] * w[k];
    }
    if (!(nn > T(1e-12))) return false;
    const T inv = T(1) / PM<T>::sqrt_(nn);
    for (int k = 0; k < 3; k++) u[k] = w[k] * inv;
  }
  T lo[3] = {T(1e30), T(1e30), T(1e30)}, hi[3] = {T(-1e30), T(-1e30), T(-1e30)};
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int i = 64 * j + l;
    if (i < n) {
      const T* V = m.mesh_vert[vadr + i];
      T d[3];
      for (int k = 0; k < 3; k++) d[k] = s.gpos[gm][k] + Rm[3 * k] * V[0] + Rm[3 * k + 1] * V[1] + Rm[3 * k + 2] * V[2] - s.gpos[gb][k];
      if (sph) {
        const T t = u[0] * d[0] + u[1] * d[1] + u[2] * d[2];
        lo[0] = fmin(lo[0], t);
      } else {
        for (int k = 0; k < 3; k++) {
          const T q = Rb[k] * d[0] + Rb[3 + k] * d[1] + Rb[6 + k] * d[2] - cb[k];   // (Rb^T d)_k - centre_k
          lo[k] = fmin(lo[k], q);
          hi[k] = fmax(hi[k], q);
        }
      }
    }
  }
  const T mg = margin + T(1e-5);
  if (sph) return -c_wave_max(-lo[0]) > m.geom_size[gb][0] + mg;
  bool sep = false;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T h = cb[3 + k] + mg;
    sep = sep || -c_wave_max(-lo[k]) > h || c_wave_max(hi[k]) < -h;
  }
  return sep;
}
template <typename T>
__device__ bool c_convex_screen(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2, T margin) {
  const DevPhys<T>& m = phys<T>();
  // (convex pairs: g2 a mesh, g1 a sphere, box or mesh)
  if (c_hull_beyond(m, s, g2, g1, margin)) return true;
  return m.geom_type[g1] == 7 && c_hull_beyond(m, s, g1, g2, margin);
}

// broadphase pre-test: geom gs's bounding sphere (centre gpos, radius rbound -- MuJoCo's) does not
// reach geom gb's bounding box (geom_aabb in gb's frame) inflated by the margin.  Exact cull:
// every point of gs lies in its sphere and every point of gb in its box, so a pair culled here
// has no two points within the margin.
template <typename T>
__device__ __forceinline__ bool c_sphere_obb_disjoint(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int gs, int gb, T margin) {
  const DevPhys<T>& m = phys<T>();
  const T* R = s.gmat[gb];
  const T* c = m.geom_aabb[gb];
  const T d[3] = {s.gpos[gs][0] - s.gpos[gb][0], s.gpos[gs][1] - s.gpos[gb][1], s.gpos[gs][2] - s.gpos[gb][2]};
  T q = 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T loc = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2] - c[k];   // (R^T d)_k - centre_k
    const T out = fmax(fabs(loc) - c[3 + k], T(0));
    q += out * out;
  }
  const T r = m.geom_rbound[gs] + margin;
  return q > r * r;
}

// plane pairs: the other geom's oriented bounding box lies entirely beyond the plane (by more
// than the margin, plus 1 um of slack) -- no vertex / corner / surface point can reach it, so the
// pair cannot produce a contact.  Exact cull: the contact set is unchanged.
template <typename T>
__device__ __forceinline__ bool c_plane_obb_clear(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int gp, int g, T margin) {
  const DevPhys<T>& m = phys<T>();
  const T* Rp = s.gmat[gp];
  const T n[3] = {Rp[2], Rp[5], Rp[8]};
  const T* R = s.gmat[g];
  const T* c = m.geom_aabb[g];
  T d = 0, ext = 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T ck = s.gpos[g][k] + R[3 * k] * c[0] + R[3 * k + 1] * c[1] + R[3 * k + 2] * c[2];
    d += n[k] * (ck - s.gpos[gp][k]);
    ext += c[3 + k] * fabs(n[0] * R[k] + n[1] * R[3 + k] + n[2] * R[6 + k]);
  }
  return d - ext > margin + T(1e-6);
}

template <typename T>
__device__ void t_makeframe(T f[9]) {
  t_normalize3(f);
  if (PM<T>::sqrt_(f[3] * f[3] + f[4] * f[4] + f[5] * f[5]) < T(0.5)) {
    if (fabs(f[1]) < T(0.5)) { f[3] = 0; f[4] = 1; f[5] = 0; }
    else { f[3] = 0; f[4] = 0; f[5] = 1; }
  }
  const T d = f[0] * f[3] + f[1] * f[4] + f[2] * f[5];
  f[3] -= f[0] * d; f[4] -= f[1] * d; f[5] -= f[2] * d;
  t_normalize3(f + 3);
  t_cross(f + 6, f, f + 3);
}

// mjc_Convex (oracle/convex.c): MPR (the OBB pre-test ran in the broadphase), mjc_fixNormal for the
// sphere, and with multiccd (shelf_pnp.xml:5) four more MPR runs with the geoms rotated in opposite
// senses by +-1e-3 rad about the first contact's tangent axes; a contact farther than 1e-3 x
// min(rbound) from the pair's earlier ones is added.  Up to C_MULTI contacts, staged at val[0 ..)
// (dist, pos, normal) by lane 0; returns their number.  Wave-uniform call: every lane passes the
// same pair and gets the same result.
constexpr int C_MULTI = 5;
template <typename T, int G>
__device__ __forceinline__ bool c_mpr_contact(const DevPhys<T>& /*image: phys<T>()*/, const CShape<T, G>* sh, T margin,
                                              T* c, double (*sv)[6]) {
  const DevPhys<T>& m = phys<T>();
  CT depth, nrm[3], pos[3];
#if PNP_MPR_SLOTS
  if (!c_mpr<T, SVertL, G>(m, sh[0], sh[1], depth, nrm, pos, sv)) return false;
#else
  (void)sv;
  if (!c_mpr(m, sh[0], sh[1], depth, nrm, pos)) return false;
#endif
  if (nrm[0] == 0 && nrm[1] == 0 && nrm[2] == 0) return false;   // normal undefined
  if (sh[0].type == 2) {   // mjc_fixNormal: the sphere's normal at the contact point (g1 of its pairs)
    CT n[3];
    cs3(n, pos, sh[0].pos);
    const CT len = PM<CT>::sqrt_(cd3(n, n));
    if (len < CT(1e-15)) { nrm[0] = 1; nrm[1] = 0; nrm[2] = 0; }
    else { nrm[0] = n[0] / len; nrm[1] = n[1] / len; nrm[2] = n[2] / len; }
  }
  c[0] = T(CT(margin) - depth);
  for (int k = 0; k < 3; k++) { c[1 + k] = T(pos[k]); c[4 + k] = T(nrm[k]); }
  return true;
}
// A geom's world frame for the colliders, in CT.  fp32 builds (PNP_XLO): the position from the
// body's fp32 pair xpos + xlo (the fp64 kinematic chain's position) plus the body frame times the
// geom offset, in CT; the rotation (MPR) from xquat + xqlo, the chain's quaternion, where the
// build keeps it (PNP_XQLO), else gmat -- not the geom's fp32 gpos / gmat, rounded at world scale
// (~3e-8 m at 1 m) and per body (~6e-8 rad).  fp64: gpos / gmat.  R may be null (position only).
template <typename T>
__device__ __forceinline__ void c_geom_frame64(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g, CT* pos,
                                               CT* R) {
#if PNP_XLO
  if constexpr (sizeof(T) == 4) {
    const DevPhys<T>& m = phys<T>();
    const int b = m.geom_bodyid[g];
    const T* Rb = s.xmat[b];
    const T* gp = m.geom_pos[g];
#pragma unroll
    for (int k = 0; k < 3; k++)
      pos[k] = (CT(s.xpos[b][k]) + CT(s.xlo[b][k])) +
               (CT(Rb[3 * k]) * CT(gp[0]) + CT(Rb[3 * k + 1]) * CT(gp[1]) + CT(Rb[3 * k + 2]) * CT(gp[2]));
    if (R) {
#if PNP_XQLO
      CT q[4], gq[4], qg[4];
#pragma unroll
      for (int k = 0; k < 4; k++) { q[k] = CT(s.xquat[b][k]) + CT(s.xqlo[b][k]); gq[k] = CT(m.geom_quat[g][k]); }
      d_mulquat(qg, q, gq);
      d_quat2mat(R, qg);
#else
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = CT(s.gmat[g][k]);
#endif
    }
    return;
  }
#endif
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = CT(s.gpos[g][k]);
  if (R)
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = CT(s.gmat[g][k]);
}
// geom g2's centre relative to g1's: in fp32 builds the difference of the two fp64 centres
// (c_geom_frame64) rounded once -- the relative position of two bodies near each other (closed
// finger pads, a cube in the fingers), not the difference of two world positions each rounded at
// ~1 m (~6e-8 m: ~300 times the fp32 resolution of a finger's slide joint; the one-ulp
// conditioning floor of the closed-finger fixture is 5e-5 and pad-pad contacts turned that
// rounding into 1.6e-4, round 4); fp64: gpos[g2] - gpos[g1]
template <typename T>
__device__ __forceinline__ void c_rel_pos(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2, T* d) {
#if PNP_XLO
  if constexpr (sizeof(T) == 4) {
    const DevPhys<T>& m = phys<T>();
    CT o1[3], o2[3];
    c_geom_frame64(m, s, g1, o1, (CT*)nullptr);
    c_geom_frame64(m, s, g2, o2, (CT*)nullptr);
#pragma unroll
    for (int k = 0; k < 3; k++) d[k] = T(o2[k] - o1[k]);
    return;
  }
#endif
#pragma unroll
  for (int k = 0; k < 3; k++) d[k] = s.gpos[g2][k] - s.gpos[g1][k];
}
// the pair's two shapes, origin at geom 1's centre (oracle/convex.c): centimetre-scale support
// points, so the fp32 Minkowski differences keep ~20x more bits than in world coordinates
template <typename T, int G>
__device__ __forceinline__ void c_convex_shapes(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2,
                                                T margin, CShape<T, G>* sh) {
  const DevPhys<T>& m = phys<T>();
  const int gs[2] = {g1, g2};
  CT o1[3], o2[3];
  c_geom_frame64(m, s, g1, o1, sh[0].R);
  c_geom_frame64(m, s, g2, o2, sh[1].R);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int g = gs[i];
    sh[i].type = m.geom_type[g];
    sh[i].mesh = m.geom_dataid[g];
    sh[i].margin = margin;
    for (int k = 0; k < 3; k++) { sh[i].pos[k] = i == 0 ? CT(0) : o2[k] - o1[k]; sh[i].size[k] = m.geom_size[g][k]; }
    c_load_shape(m, sh[i]);
  }
}
// multiccd trial t (0..3): geom 1 rotated by q, geom 2 by q^-1, both about the first contact's
// position o (mjc_rotateFrame; an unverified assumption, oracle/convex.c), q the rotation by
// a = -+1e-3 rad about the first contact's tangent axis t >> 1 (frame f = mju_makeFrame of its
// normal): q = (cos(a/2), axis sin(a/2)) (oracle: sp_axisangle2quat), R(q^-1) = R(q)^T.  sh[].pos
// and sh[].R hold the unperturbed frames on entry (c_convex_shapes).
// (One function for the serial and the multi-wave convex passes: same bits.)
template <typename T, int G>
__device__ __forceinline__ void c_fan_rotate(CShape<T, G>* sh, const CT* f, const CT* o, int t) {
  const bool second = (t >> 1) != 0;   // (selects, not an index: f stays in registers)
  const CT ax[3] = {second ? f[6] : f[3], second ? f[7] : f[4], second ? f[8] : f[5]};
  const CT sh_ = (t & 1) ? CT(0.0004999999791666669) : CT(-0.0004999999791666669), q0 = CT(0.9999998750000026);
  const CT q[4] = {q0, ax[0] * sh_, ax[1] * sh_, ax[2] * sh_};
  CT Rq[9];
  const CT q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  const CT q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  const CT q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  Rq[0] = q00 + q11 - q22 - q33; Rq[4] = q00 - q11 + q22 - q33; Rq[8] = q00 - q11 - q22 + q33;
  Rq[1] = 2 * (q12 - q03); Rq[2] = 2 * (q13 + q02); Rq[3] = 2 * (q12 + q03);
  Rq[5] = 2 * (q23 - q01); Rq[6] = 2 * (q13 - q02); Rq[7] = 2 * (q23 + q01);
  CT Ra[9], Rb[9];
#pragma unroll
  for (int k = 0; k < 9; k++) { Ra[k] = sh[0].R[k]; Rb[k] = sh[1].R[k]; }
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      sh[0].R[3 * i + j] = Rq[3 * i] * Ra[j] + Rq[3 * i + 1] * Ra[3 + j] + Rq[3 * i + 2] * Ra[6 + j];
      sh[1].R[3 * i + j] = Rq[i] * Rb[j] + Rq[3 + i] * Rb[3 + j] + Rq[6 + i] * Rb[6 + j];
    }
  CT r0[3], r1[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { r0[k] = sh[0].pos[k] - o[k]; r1[k] = sh[1].pos[k] - o[k]; }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    sh[0].pos[k] = o[k] + (Rq[3 * k] * r0[0] + Rq[3 * k + 1] * r0[1] + Rq[3 * k + 2] * r0[2]);
    sh[1].pos[k] = o[k] + (Rq[k] * r1[0] + Rq[3 + k] * r1[1] + Rq[6 + k] * r1[2]);
  }
}
// the perturbation frame from the first contact's normal n0
template <typename T>
__device__ __forceinline__ void c_fan_frame(const T* n0, CT* f) {
  f[0] = n0[0]; f[1] = n0[1]; f[2] = n0[2];
  for (int k = 3; k < 9; k++) f[k] = 0;
  t_makeframe(f);
}
// distinct-contact tolerance (relative_tolerance x min rbound) and test (positions of one frame)
template <typename T>
__device__ __forceinline__ T c_fan_tol(const DevPhys<T>& /*image: phys<T>()*/, int g1, int g2) {
  const DevPhys<T>& m = phys<T>();
  return T(1e-3) * fmin(m.geom_rbound[g1], m.geom_rbound[g2]);
}
template <typename T>
__device__ __forceinline__ bool c_fan_close(const T* a, const T* b, T tol) {
  const T e[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  return PM<T>::sqrt_(cd3(e, e)) <= tol;
}
// One MPR run of the pair (g1, g2): the first (t = -1) or multiccd trial t (the perturbation frame
// from val[0]'s normal, the pair's staged first contact); lane 0 stages the contact (position
// relative to geom 1's centre) at val[slot].  Wave-uniform result.  One call site per pass: with
// the first run and the trials at two call sites, the convex stage's spills grew the compact
// build's scratch 304 -> 896 B per lane and cost C3 2 % although C3 never runs the stage (392 B and
// -1.0 % with one).  The serial and the multi-wave convex passes both call it: the same bits.
#if PNP_MW
#define C_RUN_INLINE __attribute__((noinline))   // two call sites (serial and multi-wave passes)
#else
#define C_RUN_INLINE __forceinline__              // one call site (c_convex's loop)
#endif
// G = 16: every argument is the lane group's own (four runs per wave, step.hip convex_part); the
// group's first lane stages the contact
template <typename T, int G = 64>
__device__ C_RUN_INLINE bool c_convex_run(const Env<T>& s, int g1, int g2, T margin, int t, T (*val)[7], int slot) {
  const DevPhys<T>& m = phys<T>();
  CShape<T, G> sh[2];
  c_convex_shapes(m, s, g1, g2, margin, sh);
  if (t >= 0) {
    CT f[9];
    c_fan_frame(val[0] + 4, f);
    const CT o[3] = {CT(val[0][1]), CT(val[0][2]), CT(val[0][3])};   // first contact (geom-1-centred)
    c_fan_rotate(sh, f, o, t);
  }
  T c[7];
#if PNP_MPR_SLOTS
  // this group's portal slots
  double (*sv)[6] = const_cast<Env<T>&>(s).mpr_sv[threadIdx.x >> 6][(threadIdx.x & 63) / G];
#else
  double (*sv)[6] = nullptr;
#endif
  const bool hit = c_mpr_contact(m, sh, margin, c, sv);
  if (hit && (threadIdx.x & (G - 1)) == 0)
    for (int k = 0; k < 7; k++) val[slot][k] = c[k];
  return hit;
}
template <typename T>
__device__ __forceinline__ int c_convex(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2, T margin,
                                        T (*val)[7]) {
  const DevPhys<T>& m = phys<T>();
  const int l = threadIdx.x & 63;
  // (the compact build runs the first MPR only: step.hip); smooth geoms (the sphere, always g1 of its
  // pairs) make no fan (oracle/convex.c mpr_fan)
  const int trips = (!PNP_COMPACT && m.multiccd && m.geom_type[g1] != 2 && m.geom_type[g2] != 2) ? 4 : 0;
  int n = 0;
  for (int t = -1; t < trips; t++) {   // t = -1: the first run; then the multiccd trials
    wsync();
    if (!c_convex_run(s, g1, g2, margin, t, val, n)) {
      if (t < 0) return 0;
      continue;
    }
    wsync();
    bool distinct = true;
    const T tol = c_fan_tol(m, g1, g2);
    for (int i = 0; i < n; i++)
      if (c_fan_close(val[n] + 1, val[i] + 1, tol)) distinct = false;
    if (distinct) n++;
  }
  wsync();
  if (l == 0) {
    CT o1[3];
    c_geom_frame64(m, s, g1, o1, (CT*)nullptr);
    for (int i = 0; i < n; i++)
      for (int k = 0; k < 3; k++) val[i][1 + k] = T(CT(val[i][1 + k]) + o1[k]);
  }
  wsync();
  return n;
}

template <typename T>
__device__ void c_params(const DevPhys<T>& /*image: phys<T>()*/, Con<T>& c, int g1, int g2) {
  const DevPhys<T>& m = phys<T>();
  t_makeframe(c.frame);
  c.g1 = g1;
  c.g2 = g2;
  c.dim = max(m.geom_condim[g1], m.geom_condim[g2]);
  if (m.geom_priority[g1] != m.geom_priority[g2]) c.dim = m.geom_priority[g1] > m.geom_priority[g2] ? m.geom_condim[g1] : m.geom_condim[g2];
  T f[3];
  for (int k = 0; k < 3; k++) f[k] = fmax(m.geom_friction[g1][k], m.geom_friction[g2][k]);
  c.friction[0] = c.friction[1] = f[0];
  c.friction[2] = f[1];
  c.friction[3] = c.friction[4] = f[2];
  const T s1 = m.geom_solmix[g1], s2 = m.geom_solmix[g2];
  T mix;
  if (s1 >= T(1e-15) && s2 >= T(1e-15)) mix = s1 / (s1 + s2);
  else if (s1 < T(1e-15) && s2 < T(1e-15)) mix = T(0.5);
  else mix = s1 < T(1e-15) ? T(0) : T(1);
  if (m.geom_solref[g1][0] > 0 && m.geom_solref[g2][0] > 0)
    for (int k = 0; k < 2; k++) c.solref[k] = mix * m.geom_solref[g1][k] + (1 - mix) * m.geom_solref[g2][k];
  else
    for (int k = 0; k < 2; k++) c.solref[k] = fmin(m.geom_solref[g1][k], m.geom_solref[g2][k]);
  for (int k = 0; k < 5; k++) c.solimp[k] = mix * m.geom_solimp[g1][k] + (1 - mix) * m.geom_solimp[g2][k];
  c.includemargin = fmax(m.geom_margin[g1], m.geom_margin[g2]) - fmax(m.geom_gap[g1], m.geom_gap[g2]);
}

template <typename T, class S>
__device__ void collide_geoms(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int g1, int g2, S& out) {
  const DevPhys<T>& m = phys<T>();
  const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
  const T *p1 = s.gpos[g1], *R1 = s.gmat[g1], *s1 = m.geom_size[g1];
  const T *p2 = s.gpos[g2], *R2 = s.gmat[g2], *s2 = m.geom_size[g2];
  const T margin = fmax(m.geom_margin[g1], m.geom_margin[g2]);
  if (t1 == 0 && t2 == 2) c_plane_sphere(p1, R1, p2, s2[0], margin, out);
  else if (t1 == 0 && t2 == 6) c_plane_box(p1, R1, p2, R2, s2, margin, out);
  else if (t1 == 0 && t2 == 7) c_plane_mesh(m, p1, R1, p2, R2, m.geom_dataid[g2], margin, out);
  else if (t1 == 2 && t2 == 2) c_sphere_sphere(p1, s1[0], p2, s2[0], margin, out);
  else if (t1 == 2 && t2 == 6) c_sphere_box(p1, s1[0], p2, R2, s2, margin, out);
  else if (t1 == 6 && t2 == 6) {
    T Tv[3];   // box 2's centre relative to box 1's
    c_rel_pos(m, s, g1, g2, Tv);
    c_box_box(p1, R1, s1, p2, R2, s2, Tv, margin, out);
  }
  // convex pairs: st_collision's MPR pass
}
template <typename T, class S>
__device__ __forceinline__ void collide_pair(const DevPhys<T>& /*image: phys<T>()*/, const Env<T>& s, int pair, S& out) {
  const DevPhys<T>& m = phys<T>();
  collide_geoms(m, s, m.pair_g1[pair], m.pair_g2[pair], out);
}
