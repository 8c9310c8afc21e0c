// Device-side trace loop for gfx950 (included by trace.hip only).
//
// One lane = one pixel; its samples are traced sequentially so the per-pixel
// sum keeps the reference's accumulation order (myScene.java:1451-1460).
// Geometry and shading are IEEE fp64 with the reference's expression order
// (compiled -ffp-contract=off, no fast-math) so that every discrete decision
// (hit object, shadow, TIR) matches the oracle; see DESIGN.md "Precision".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_types.h"
#define QD_FN __device__ __forceinline__
#include "qdiv.h"

namespace rt {
namespace dv {

#define DEVI __device__ __forceinline__

static constexpr double EPS = 0.0000001;
static constexpr double DMAX = 1.7976931348623157e308;
static constexpr double TWO_PI_F = 6.2831854820251465;   // (double)PConstants.TWO_PI
static constexpr double PI_F = 3.1415927410125732;       // (double)PConstants.PI
static constexpr double PI_D = 3.141592653589793;        // Math.PI

enum : uint32_t {
  SITE_AA_Y = 1, SITE_AA_X = 2, SITE_DOF_ANG = 3, SITE_DOF_RAD = 4, SITE_TIME = 8,
  SITE_DISK = 0x100, SITE_SHADOW_TIME = 0x200, SITE_PH_DIR = 0x1000, SITE_PH_BOUNCE = 0x1100, SITE_PH_TIME = 0x1200
};
enum { C_CAMERA = 0, C_SHADOW, C_REFL, C_REFR, C_BOX, C_TRI, C_QUAD, C_IMPLICIT, C_LIGHT, C_PHOTON, C_TEXEL,
       C_NODE, C_LEAF, C_MEMBER, C_ROOT, C_TOP,
       // record loads per wave step (include/distraytracer.h RT_ST_W_*)
       C_WNODE, C_WTRI, C_WQUAD, C_WIMPLICIT, C_WLIGHT, C_WPHOTON, C_N = 24 };

struct V {
  double x, y, z;
};
DEVI V mk(double x, double y, double z) { V r; r.x = x; r.y = y; r.z = z; return r; }
DEVI V sub(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEVI V add(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEVI V scl(V a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
DEVI double dot(V a, V b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
DEVI V cross(V a, V b) { return mk((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)); }
DEVI double mag(V a) { return sqrt(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z)); }
DEVI V nrmz(V a) {  // myVector._normalize: division, no-op on zero
  double m = mag(a);
  if (m == 0) return a;
  return mk(a.x / m, a.y / m, a.z / m);
}
DEVI bool veq(V a, V b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
DEVI V ld3(const double* p) { return mk(p[0], p[1], p[2]); }
DEVI double jmin(double a, double b) { return (a != a) ? a : ((a <= b) ? a : b); }  // Math.min (finite paths)
DEVI double jmax(double a, double b) { return (a != a) ? a : ((a >= b) ? a : b); }
DEVI int32_t jd2i(double v) {
  if (v != v) return 0;
  if (v >= 2147483647.0) return 2147483647;
  if (v <= -2147483648.0) return (int32_t)0x80000000;
  return (int32_t)v;
}
// myMatrix.multVert: accumulate from 0 in column order (keeps signed-zero behaviour)
DEVI V xpt(const double* m, V p) {
  double r[3];
#pragma unroll
  for (int row = 0; row < 3; ++row) {
    double a = 0.0;
    a += m[row * 4 + 0] * p.x;
    a += m[row * 4 + 1] * p.y;
    a += m[row * 4 + 2] * p.z;
    a += m[row * 4 + 3] * 1.0;
    r[row] = a;
  }
  return mk(r[0], r[1], r[2]);
}
DEVI V xvec(const double* m, V p) {
  double r[3];
#pragma unroll
  for (int row = 0; row < 3; ++row) {
    double a = 0.0;
    a += m[row * 4 + 0] * p.x;
    a += m[row * 4 + 1] * p.y;
    a += m[row * 4 + 2] * p.z;
    a += m[row * 4 + 3] * 0.0;
    r[row] = a;
  }
  return mk(r[0], r[1], r[2]);
}

// keyed counter RNG (same definition as the oracle's; DESIGN.md "RNG")
DEVI uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
DEVI double rng(uint64_t seed, uint64_t a, uint32_t b, uint32_t c, uint32_t site, uint32_t k, double lo, double hi) {
  uint64_t h = mix64(seed ^ mix64(a));
  h = mix64(h ^ (((uint64_t)b << 32) | c));
  h = mix64(h ^ (((uint64_t)site << 32) | k));
  double r = (double)(h >> 11) * 0x1.0p-53;
  r = r * (hi - lo) + lo;
  if (r >= hi) r = __longlong_as_double(__double_as_longlong(hi) - 1);
  return r;
}

// RNG key of the ray currently traced
struct Key {
  uint64_t seed, pixel;
  uint32_t sample, node;
  uint32_t tsite;  // RNG site of per-object ray times (myRay.getTime): camera/secondary, shadow or photon rays
};

// World ray with the reference's in-place re-normalisation state
// (myRay.getTransformedRay normalises the source direction, myRay.java:91-93).
// `ver` counts the re-normalisations that changed d, so the direction seen by any
// earlier test is nrmz^ver(d0) and hit candidates need not carry a direction.
struct WRay {
  V o, d, d0;
  uint32_t ver;
  bool stable;  // normalize(d) == d
  bool moved;   // d changed since the cached accel-space ray was built
};
DEVI void renorm(WRay& r) {
  if (!r.stable) {
    V n = nrmz(r.d);
    r.stable = veq(n, r.d);
    if (!r.stable) { r.moved = true; r.ver++; }
    r.d = n;
  }
}

#ifdef RT_PROF_PKSTAT  // profiling builds only (tools/pkstat.py): packet-traversal lane utilisation
// wave steps and the lanes testing in them: closest box / triangle, any-hit box / triangle
// + closest-hit calls of the shading tree (one per traced camera / secondary ray) and shadow-ray calls
enum { P_CB_STEP = C_N, P_CB_LANES, P_CT_STEP, P_CT_LANES, P_AB_STEP, P_AB_LANES, P_AT_STEP, P_AT_LANES,
       P_RAY_STEP, P_RAY_LANES, P_SH_STEP, P_SH_LANES,
       P_CTH_STEP, P_CTH_LANES, P_ATH_STEP, P_ATH_LANES,  // triangle wave steps with a hitting lane
       P_N };
#else
enum { P_N = C_N };
#endif
struct Counters {
  uint64_t c[P_N];
};

// ---------------------------------------------------------------------------
// primitive tests (object space). `args` carries what the hit record needs:
// planar orientation, cylinder face, box plane.
struct RayInv {
  double y[3];  // RN(1 / d_i)
  bool fast;    // qdiv is exact for this ray (see qdiv)
};
DEVI RayInv ray_inv(V o, V d, int sceneOk) {
  RayInv r;
  r.y[0] = 1.0 / d.x; r.y[1] = 1.0 / d.y; r.y[2] = 1.0 / d.z;
  r.fast = sceneOk && qd_range(d.x) && qd_range(d.y) && qd_range(d.z) && qc_range(o.x) && qc_range(o.y) && qc_range(o.z);
  return r;
}

template <bool FAST>
DEVI bool slab_t(const double* mn, const double* mx, V o, V d, const double* y, double& tEntry) {  // myBBox.intersectCheck :132-162
  double ro[3] = {o.x, o.y, o.z}, rd[3] = {d.x, d.y, d.z};
  double tMin[3], tMax[3];
  double biggestMin = -DMAX;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double t1 = FAST ? qdiv(mn[i] - ro[i], rd[i], y[i]) : (mn[i] - ro[i]) / rd[i];
    double t2 = FAST ? qdiv(mx[i] - ro[i], rd[i], y[i]) : (mx[i] - ro[i]) / rd[i];
    if (t1 < t2) {
      tMin[i] = t1; tMax[i] = t2;
      if (biggestMin < t1) biggestMin = t1;
    } else {
      tMin[i] = t2; tMax[i] = t1;
      if (biggestMin < t2) biggestMin = t2;
    }
  }
  double mnv = DMAX, mxv = -DMAX;  // p.min / p.max skip NaN
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (tMax[i] < mnv) mnv = tMax[i];
    if (tMin[i] > mxv) mxv = tMin[i];
  }
  tEntry = biggestMin;
  return (mnv > mxv) && biggestMin > 0;
}
DEVI bool slab(const double* mn, const double* mx, V o, V d, double& tEntry) {
  return slab_t<false>(mn, mx, o, d, nullptr, tEntry);
}
// ---- box tests on the traversal hot path --------------------------------------------
// With a valid RayInv (ri.fast) every slab t is first approximated as t' = RN(a * y),
// within 2^-51 |t'| of the exact t = RN(a / b) (a = RN(bound - o) as in the exact test).
// The box decisions only compare slab values (with each other, with 0, with a hit t or a
// shadow distance), so t' settles a decision whenever the compared quantities are further
// apart than a 2^-46 relative margin; otherwise (grazing rays) the exact test decides.
// The sign of every t' equals the sign of t (no underflow in the qdiv ranges), so
// "entry > 0" is always settled exactly.
static constexpr double APX = 0x1p-46;
DEVI int slab_apx(const double* mn, const double* mx, V o, const double* y, double& lo) {
  const double b0 = mn[0], b1 = mn[1], b2 = mn[2], b3 = mx[0], b4 = mx[1], b5 = mx[2];
  const double t0 = (b0 - o.x) * y[0], t3 = (b3 - o.x) * y[0];
  const double t1 = (b1 - o.y) * y[1], t4 = (b4 - o.y) * y[1];
  const double t2 = (b2 - o.z) * y[2], t5 = (b5 - o.z) * y[2];
  lo = fmax(fmax(fmin(t0, t3), fmin(t1, t4)), fmin(t2, t5));
  const double hi = fmin(fmin(fmax(t0, t3), fmax(t1, t4)), fmax(t2, t5));
  if (!(lo > 0)) return 0;
  const double diff = hi - lo, tol = APX * (fabs(hi) + fabs(lo));
  if (diff > tol) return 1;
  if (-diff > tol) return 0;
  return -1;
}
// The same approximate test as two masks instead of a tri-state int (RT_APX2): `sure` -- the box
// decision is settled (a miss, or a hit / miss beyond the margin); the return value -- a settled hit.
// The compares feed the branch as lane masks; the int's selects and re-compares are gone.
#ifndef RT_APX2
#define RT_APX2 0
#endif
DEVI bool slab_apx2(const double* mn, const double* mx, V o, const double* y, double& lo, bool& sure) {
  const double b0 = mn[0], b1 = mn[1], b2 = mn[2], b3 = mx[0], b4 = mx[1], b5 = mx[2];
  const double t0 = (b0 - o.x) * y[0], t3 = (b3 - o.x) * y[0];
  const double t1 = (b1 - o.y) * y[1], t4 = (b4 - o.y) * y[1];
  const double t2 = (b2 - o.z) * y[2], t5 = (b5 - o.z) * y[2];
  lo = fmax(fmax(fmin(t0, t3), fmin(t1, t4)), fmin(t2, t5));
  const double hi = fmin(fmin(fmax(t0, t3), fmax(t1, t4)), fmax(t2, t5));
  const bool pos = lo > 0;
  const double diff = hi - lo, tol = APX * (fabs(hi) + fabs(lo));
  const bool in = diff > tol;
  sure = !pos || in || (-diff > tol);
  return pos && in;
}
DEVI bool slab_exact(const double* mn, const double* mx, V o, V d, const RayInv& ri, double& tEntry) {
  if (ri.fast) return slab_t<true>(mn, mx, o, d, ri.y, tEntry);
  return slab_t<false>(mn, mx, o, d, nullptr, tEntry);
}
// hit?  (myBBox.intersectCheck != null)
template <bool A2 = (RT_APX2 != 0)>  // A2: slab_apx2 (lane masks)
DEVI bool box_hit(const double* mn, const double* mx, V o, V d, const RayInv& ri) {
  double te;
  if (A2 && ri.fast) {
    bool sure;
    const bool h = slab_apx2(mn, mx, o, ri.y, te, sure);
    if (sure) return h;
  } else if (ri.fast) {
    int r = slab_apx(mn, mx, o, ri.y, te);
    if (r >= 0) return r != 0;
  }
  return slab_exact(mn, mx, o, d, ri, te);
}
// hit and (lim == DMAX or entry t < lim)   (BVH right-child rule)
template <bool A2 = (RT_APX2 != 0)>  // A2: slab_apx2 (lane masks)
DEVI bool box_before(const double* mn, const double* mx, V o, V d, const RayInv& ri, double lim) {
  double te;
  if (A2 && ri.fast) {
    bool sure;
    const bool h = slab_apx2(mn, mx, o, ri.y, te, sure);
    if (sure) {
      if (!h) return false;
      if (lim == DMAX) return true;
      const double tol = APX * (fabs(te) + fabs(lim));
      if (lim - te > tol) return true;
      if (te - lim > tol) return false;
    }
  } else if (ri.fast) {
    int r = slab_apx(mn, mx, o, ri.y, te);
    if (r == 0) return false;
    if (r == 1) {
      if (lim == DMAX) return true;
      const double tol = APX * (fabs(te) + fabs(lim));
      if (lim - te > tol) return true;
      if (te - lim > tol) return false;
    }
  }
  if (!slab_exact(mn, mx, o, d, ri, te)) return false;
  return lim == DMAX || te < lim;
}
// hit and dist - entry t > 1e-7   (calcShadowHit on a box)
template <bool A2 = (RT_APX2 != 0)>  // A2: slab_apx2 (lane masks)
DEVI bool box_shadow(const double* mn, const double* mx, V o, V d, const RayInv& ri, double dist) {
  double te;
  if (A2 && ri.fast) {
    bool sure;
    const bool h = slab_apx2(mn, mx, o, ri.y, te, sure);
    if (sure) {
      if (!h) return false;
      const double g = (dist - te) - EPS, tol = APX * (fabs(te) + fabs(dist));
      if (g > tol) return true;
      if (-g > tol) return false;
    }
  } else if (ri.fast) {
    int r = slab_apx(mn, mx, o, ri.y, te);
    if (r == 0) return false;
    if (r == 1) {
      const double g = (dist - te) - EPS, tol = APX * (fabs(te) + fabs(dist));
      if (g > tol) return true;
      if (-g > tol) return false;
    }
  }
  return slab_exact(mn, mx, o, d, ri, te) && (dist - te) > EPS;
}

// box_shadow that also reports the box's entry t (approximate: the ordering of the nearest-first
// any-hit traversal, never a decision)
template <bool A2 = (RT_APX2 != 0)>  // A2: slab_apx2 (lane masks)
DEVI bool box_shadow_e(const double* mn, const double* mx, V o, V d, const RayInv& ri, double dist, double& te) {
  if (A2 && ri.fast) {
    bool sure;
    const bool h = slab_apx2(mn, mx, o, ri.y, te, sure);
    if (sure) {
      if (!h) return false;
      const double g = (dist - te) - EPS, tol = APX * (fabs(te) + fabs(dist));
      if (g > tol) return true;
      if (-g > tol) return false;
    }
  } else if (ri.fast) {
    int r = slab_apx(mn, mx, o, ri.y, te);
    if (r == 0) return false;
    if (r == 1) {
      const double g = (dist - te) - EPS, tol = APX * (fabs(te) + fabs(dist));
      if (g > tol) return true;
      if (-g > tol) return false;
    }
  }
  return slab_exact(mn, mx, o, d, ri, te) && (dist - te) > EPS;
}

DEVI int slab_plane(const double* mn, const double* mx, V o, V d) {  // plane idx for myBBox normals
  double ro[3] = {o.x, o.y, o.z}, rd[3] = {d.x, d.y, d.z};
  double biggestMin = -DMAX;
  int idx = -1;
  for (int i = 0; i < 3; ++i) {
    double t1 = (mn[i] - ro[i]) / rd[i], t2 = (mx[i] - ro[i]) / rd[i];
    if (t1 < t2) { if (biggestMin < t1) { idx = i; biggestMin = t1; } }
    else { if (biggestMin < t2) { idx = i + 3; biggestMin = t2; } }
  }
  return idx;
}

// planar: orientation with N.d < 0 (the reference flips the vertex order in place, Q5)
// Hit filters: a candidate whose t cannot change the caller's outcome may be reported as a
// miss without running the inside test (the decision it would feed is already fixed):
// closest hit -- t neither below the subtree minimum nor below the running best;
// shadow -- not (dist - t > 1e-7). LimNone: the full test (hit records, photons).
struct LimNone {
  DEVI bool ok(double) const { return true; }
};
struct LimClosest {
  double a, b;
  DEVI bool ok(double t) const { return t < a || t < b; }
};
struct LimShadow {
  double dist;
  DEVI bool ok(double t) const { return (dist - t) > EPS; }
};

template <int NV, bool PLANE, class LIM = LimNone>
DEVI bool planar_test(const double (*v)[3], V nA, V nB, double dA, double dB, V o, V d, double& t, int& st,
                      const LIM& lim = LIM()) {
  double pr = dot(nA, d);
  if (!(fabs(pr) > 0)) return false;
  V N;
  double D;
  if (pr > 0) {
    pr = dot(nB, d);
    if (!(fabs(pr) > 0) || pr > 0) return false;
    N = nB; D = dB; st = 1;
  } else {
    N = nA; D = dA; st = 0;
  }
  t = -(dot(N, o) + D) / pr;
  if (!(t > EPS)) return false;
  if (PLANE) return true;
  if (!lim.ok(t)) return false;
  V p = mk(d.x * t + o.x, d.y * t + o.y, d.z * t + o.z);
#pragma unroll
  for (int i = 0; i < NV; ++i) {  // checkInside (myPlanarObject.java:165-175, 200-211)
    int vi = st ? (NV - 1 - i) : i;
    int pi = st ? (NV - 1 - (i == 0 ? NV - 1 : i - 1)) : (i == 0 ? NV - 1 : i - 1);
    V w = ld3(v[vi]), wp = ld3(v[pi]);
    V e = sub(w, wp);
    V ir = mk(p.x - w.x, p.y - w.y, p.z - w.z);
    if (dot(cross(ir, e), N) < -EPS) return false;
  }
  return true;
}

template <class LIM = LimNone, class TR = TriD>  // TR: TriD or its geometry part (TriG)
DEVI bool tri_test(const TR& T, V o, V d, double& t, int& st, const LIM& lim = LIM()) {
  V nA = ld3(T.n);
  V nB = mk(-nA.x, -nA.y, -nA.z);  // exactly the reversed-order normal
  return planar_test<3, false>(T.v, nA, nB, T.dA, T.dB, o, d, t, st, lim);
}

// SL: the primitive record sits at a wave-uniform address (the packet kernels' top-level scans) and
// is read with scalar loads into SGPRs instead of one vector load per lane (prim_test<true>)
template <bool SL, class T>
DEVI T pld(const T* p) {
  if constexpr (SL) return *(const __attribute__((address_space(4))) T*)p;
  else return *p;
}
template <bool SL>
DEVI V pld3(const double* p) { return mk(pld<SL>(p), pld<SL>(p + 1), pld<SL>(p + 2)); }

template <bool SL = false>
DEVI V sphere_center(const PrimD& P, const Key& k) {
  if (pld<SL>(&P.type) != PT_MSPHERE) return pld3<SL>(P.a);
  // myMovingSphere.getOrigin(ray.getTime()) : keyed per (ray, object)
  double tm = rng(k.seed, k.pixel, k.sample, k.node, k.tsite, pld<SL>(&P.key), 0, 1.0);
  V o0 = pld3<SL>(P.a), o1 = pld3<SL>(P.a + 6);
  V bMa = sub(o1, o0);
  return mk(o0.x + tm * bMa.x, o0.y + tm * bMa.y, o0.z + tm * bMa.z);
}

template <bool SL = false>
DEVI bool prim_test(const PrimD& P, V o, V d, const Key& k, double& t, int& args) {
  const int32_t type = pld<SL>(&P.type);
  auto A = [&](int i) { return pld<SL>(P.a + i); };
  switch (type) {
    case PT_QUAD:
    case PT_PLANE: {
      if constexpr (SL) {
        double q[4][3];
#pragma unroll
        for (int i = 0; i < 12; ++i) q[i / 3][i % 3] = A(i);
        if (type == PT_PLANE)
          return planar_test<4, true>(q, pld3<SL>(P.a + 12), pld3<SL>(P.a + 15), A(18), A(19), o, d, t, args);
        return planar_test<4, false>(q, pld3<SL>(P.a + 12), pld3<SL>(P.a + 15), A(18), A(19), o, d, t, args);
      } else {
        const double(*v)[3] = (const double(*)[3])P.a;
        if (type == PT_PLANE)
          return planar_test<4, true>(v, ld3(P.a + 12), ld3(P.a + 15), P.a[18], P.a[19], o, d, t, args);
        return planar_test<4, false>(v, ld3(P.a + 12), ld3(P.a + 15), P.a[18], P.a[19], o, d, t, args);
      }
    }
    case PT_SPHERE:
    case PT_MSPHERE: {  // mySphere.intersectCheck (myImpObject.java:76-94)
      V c = sphere_center<SL>(P, k);
      double rx = A(3), ry = A(4), rz = A(5);
      double a = ((d.x / rx) * (d.x / rx)) + ((d.y / ry) * (d.y / ry)) + ((d.z / rz) * (d.z / rz));
      V pC = mk((o.x - c.x) / rx, (o.y - c.y) / ry, (o.z - c.z) / rz);
      double ta = 2 * a;
      double b = 2 * (((d.x / rx) * pC.x) + ((d.y / ry) * pC.y) + ((d.z / rz) * pC.z));
      double cc = (pC.x * pC.x) + (pC.y * pC.y) + (pC.z * pC.z) - 1;
      double discr = ((b * b) - (2 * ta * cc));
      if (discr < 0) return false;
      double d1 = sqrt(discr), t1 = (-1 * b + d1) / (ta), t2 = (-1 * b - d1) / (ta);
      double tv = jmin(t1, t2);
      if (tv < EPS) {
        tv = jmax(t1, t2);
        if (tv < EPS) return false;
      }
      if (tv != tv) return false;  // reference: NaN t is never a closest hit (TreeMap orders NaN last)
      t = tv;
      args = 0;
      return true;
    }
    case PT_CYL:
    case PT_HCYL: {
      double rx = A(3), rz = A(4), yTop = A(6), yBot = A(7);
      V org = pld3<SL>(P.a);
      double a = ((d.x / rx) * (d.x / rx)) + ((d.z / rz) * (d.z / rz));
      double px = (o.x - org.x) / rx, pz = (o.z - org.z) / rz;
      double b = 2 * (((d.x / rx) * px) + ((d.z / rz) * pz));
      double cc = (px * px) + (pz * pz) - 1;
      double discr = ((b * b) - (4 * a * cc));
      if (discr < 0) return false;
      double d1 = sqrt(discr), t1 = (-b + d1) / (2 * a), t2 = (-b - d1) / (2 * a);
      double cv = jmin(t1, t2), co = jmax(t1, t2);
      if (type == PT_HCYL) {  // myHollow_Cylinder.intersectCheck :174-192
        if (cv < -EPS) {
          double tmp = co; co = cv; cv = tmp;
          if (cv < -EPS) return false;
        }
        double y1 = o.y + (cv * d.y);
        if ((cv > EPS) && (y1 > yBot) && (y1 < yTop)) { t = cv; args = 0; return true; }
        double y2 = o.y + (co * d.y);
        if ((co > EPS) && (y2 > yBot) && (y2 < yTop)) { t = co; args = 1; return true; }
        return false;
      }
      // myCylinder.intersectCheck :259-302
      if (cv < EPS) {
        co = cv;
        cv = jmax(t1, t2);
        if (cv < EPS) return false;
      }
      bool planeRes = true;
      double pl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const double c0 = A(8 + 4 * i), c1 = A(9 + 4 * i), c2 = A(10 + 4 * i), c3 = A(11 + 4 * i);
        double den = c0 * d.x + c1 * d.y + c2 * d.z;
        if (fabs(den) > EPS) {
          double nm = c0 * o.x + c1 * o.y + c2 * o.z + c3;
          pl[i] = -nm / den;
        } else {
          pl[i] = 10000;
        }
      }
      double pltVal = jmin(pl[0], pl[1]);
      int idxVis = (pltVal == pl[0] ? 0 : 1);
      if (pltVal < 0) {
        pltVal = pl[idxVis];
        if (pltVal < EPS) planeRes = false;
      }
      double tVal, maxT = jmax(cv, co), minT = jmin(cv, co);
      if (planeRes && (((minT <= 0) && (pltVal >= -EPS) && (pltVal <= maxT)) || ((pltVal > minT) && (pltVal <= maxT)))) {
        tVal = pltVal;
      } else {
        tVal = cv;
        idxVis = 2;
      }
      double y1 = o.y + (tVal * d.y);
      if ((y1 + EPS >= yBot) && (y1 - EPS <= yTop)) { t = tVal; args = idxVis; return true; }
      return false;
    }
    case PT_BOX: {  // myRndrdBox -> myBBox.intersectCheck
      double te;
      if constexpr (SL) {
        double bx[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) bx[i] = A(i);
        if (!slab(bx, bx + 3, o, d, te)) return false;
        t = te;
        args = slab_plane(bx, bx + 3, o, d);
      } else {
        if (!slab(P.a, P.a + 3, o, d, te)) return false;
        t = te;
        args = slab_plane(P.a, P.a + 3, o, d);
      }
      return true;
    }
  }
  return false;
}

}  // namespace dv
}  // namespace rt
