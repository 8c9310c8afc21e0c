// HIP kernels (gfx950) for the reference's per-pixel / per-sample trace loop.
// Included by trace.hip only.
//
// Kernel structure: one lane per pixel (8x8 pixel tiles per 64-lane wave for
// ray coherence); per sample: camera ray -> shading tree evaluated post-order
// with an explicit per-lane frame stack (per-level myColor clamping, Q8, makes
// throughput-weighted path accumulation incorrect) -> closest hit = linear
// scan of objList with the reference-order BVH traversal -> lights with any-hit
// shadow rays -> reflection / refraction children.
//
// Every kernel is instantiated per scene-feature mask F (FT_* below): code for
// features a scene does not use is compiled out, which is what keeps register
// and scratch use (hence occupancy) low for the common configurations.
#pragma once
#include "trace_device.h"
#include "jfdlibm.h"  // sin / cos / asin / acos shared bit for bit with the oracle

namespace rt {
namespace dv {

// scene feature mask (host: scene_features())
enum : uint32_t {
  FT_PRIM = 1,    // non-triangle primitives (quad/plane/sphere/cylinder/box)
  FT_TEX = 2,     // image / noise / marble textures or a textured skydome
  FT_PHOTON = 4,  // photon map gather
  FT_TRANS = 8,   // transparent materials (Fresnel split, two children per node)
  FT_DOF = 16,    // lens / depth of field
  FT_LIGHTX = 32, // spot or disk lights
  FT_CAMX = 64,   // fisheye or orthographic camera
  FT_INST = 128,  // instances (named_object / instance / sierpinski)
  FT_PASS = 256,  // column step of a `refine` pass (rt_render_pass; never a scene feature)
  FT_CELL = 512,  // cellular `stone` textures (myCellularTexture: per-cell LCG, pow / log ROI functions)
  FT_ALL = 1023
};

static __constant__ int c_perm[256];  // one copy per translation unit (trace.hip uploads its own)
static __constant__ int c_grad3[12][3];

// ---------------------------------------------------------------------------
// a hit candidate: the world direction at test time is identified by the ray's
// re-normalisation version (WRay.ver), so no direction vector is carried around
struct Best {
  double t;
  int32_t ref;   // >= 0 tri, < 0 ~prim
  uint32_t ver;  // world-ray direction version at the winning test (at the instance entry for instance hits)
  int16_t top;   // objList index
  int16_t inAcc; // hit came from an accel structure (reCalcCTMHitNorm applies)
  int32_t inst;  // PT_INST prim the hit came through, -1 none
  uint32_t iver; // instance-ray direction version at the winning test
};
DEVI Best miss() { Best b; b.t = DMAX; b.ref = 0; b.top = -1; b.ver = 0; b.inAcc = 0; b.inst = -1; b.iver = 0; return b; }
// what a leaf records with a hit: objList entry, instance (or -1) and the world-ray version
// at the instance's entry (the traced ray's own version otherwise)
struct HitCtx {
  int32_t top, inst;
  uint32_t wver;
};

// Counting kernel: one count per wave step, by the step's first active lane -- for records
// a wave loads once for all its lanes (the C_W* counters)
#define WCNT(idx, n)                                                                      \
  do {                                                                                    \
    if (CNT && __lane_id() == (int)__builtin_ctzll(__ballot(1))) ct.c[idx] += (n);        \
  } while (0)
// Implicit primitives at a wave-uniform address (the packet kernels' top-level scans) as scalar loads
// into SGPRs: the record no longer occupies VGPRs inside C4's shadow scan, whose reloads of spilled
// values in that loop went from 21 static scratch ops to 1 (C4 469.5 -> 454.4 ms, C5 195.3 -> 195.1 ms,
// same images: profiles/r05h_sprim_ab.log). RT_SPRIM 2 = every variant, 1 = the variants without a
// photon map, 0 = none (vector loads, one per lane)
// RT_ULOAD: other wave-uniform records read in hot loops as scalar loads -- bit 0: a leaf member's
// transform inverse in the packet traversals (C3 3.069 -> 3.056 ms, C4 unchanged), bit 1: the light
// record's spot / disk fields in light_sum (C4 456 -> 476 ms: off). profiles/r05i_uload_ab.log
#ifndef RT_ULOAD
#define RT_ULOAD 1
#endif
#ifndef RT_SPRIM
#define RT_SPRIM 2
#endif
template <uint32_t F>
static constexpr bool SPRIM = RT_SPRIM == 2 || (RT_SPRIM == 1 && (F & FT_PHOTON) == 0);
// WAVE: the record address is wave-uniform (counted once per wave step), else per lane
template <bool CNT, uint32_t F, class LIM = LimNone, bool WAVE = false>
DEVI bool test_ref(const SceneD& S, int32_t ref, V o, V d, const Key& k, double& t, int& args, Counters& ct,
                   const LIM& lim = LIM()) {
  if (!(F & FT_PRIM) || ref >= 0) {
    if (CNT) ct.c[C_TRI]++;
    if (WAVE) WCNT(C_WTRI, 1); else if (CNT) ct.c[C_WTRI]++;
    return tri_test(S.tri[ref], o, d, t, args, lim);
  }
  const PrimD& P = S.prim[~ref];
  if (CNT) {
    const int c = (P.type == PT_QUAD || P.type == PT_PLANE) ? C_QUAD : C_IMPLICIT;
    ct.c[c]++;
    if (WAVE) WCNT(c + (C_WQUAD - C_QUAD), 1); else ct.c[c + (C_WQUAD - C_QUAD)]++;
  }
  return prim_test<WAVE && SPRIM<F>>(P, o, d, k, t, args);
}
template <uint32_t F>
DEVI int32_t ref_xf(const SceneD& S, int32_t ref) { return (!(F & FT_PRIM) || ref >= 0) ? S.tri[ref].xf : S.prim[~ref].xf; }

// Scalar (SMEM) loads of scene records at wave-uniform addresses: through the constant
// address space a uniform load is selected as s_load into SGPRs (the packet traversal
// below, where every lane of a wave works on the same node / triangle).
// (Field by field: an aggregate copy through the cast is turned back into global loads.)
template <class T>
DEVI T sload(const T* p) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "scalar field");
  return *(const __attribute__((address_space(4))) T*)p;
}
struct ChildBox {  // one child of a NodeD: box + reference
  double mn[3], mx[3];
  int32_t ref;
};
DEVI ChildBox sload_child(const NodeD* nd, int side) {
  ChildBox c;
  const double* b = side ? nd->rmin : nd->lmin;
#pragma unroll
  for (int i = 0; i < 3; ++i) { c.mn[i] = sload(b + i); c.mx[i] = sload(b + 3 + i); }
  c.ref = sload(side ? &nd->right : &nd->left);
  return c;
}
struct TriG {  // the part of a TriD the triangle test reads
  double v[3][3];
  double n[3];
  double dA, dB;
};
DEVI TriG sload_tri(const TriD* t) {
  TriG g;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int c = 0; c < 3; ++c) g.v[i][c] = sload(&t->v[i][c]);
#pragma unroll
  for (int c = 0; c < 3; ++c) g.n[c] = sload(&t->n[c]);
  g.dA = sload(&t->dA);
  g.dB = sload(&t->dB);
  return g;
}
DEVI void sload_inv(const XformD* x, double* m) {  // rows 0..2 of a CTM inverse (all multVert reads)
#pragma unroll
  for (int i = 0; i < 12; ++i) m[i] = sload(x->inv + i);
}
DEVI AccelD sload_accel(const AccelD* p) {
  AccelD a;
#pragma unroll
  for (int c = 0; c < 3; ++c) { a.bmin[c] = sload(p->bmin + c); a.bmax[c] = sload(p->bmax + c); }
  a.xf = sload(&p->xf); a.root = sload(&p->root); a.is_list = sload(&p->is_list); a.flags = sload(&p->flags);
  return a;
}
DEVI TopD sload_top(const TopD* p) {
  TopD t;
  t.kind = sload(&p->kind); t.idx = sload(&p->idx); t.xf = sload(&p->xf); t.key = sload(&p->key);
  return t;
}
DEVI int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEVI uint64_t uni64(uint64_t v) {
  return ((uint64_t)(uint32_t)uni((int32_t)(v >> 32)) << 32) | (uint32_t)uni((int32_t)(uint32_t)v);
}
// this lane's bit of a wave-uniform lane mask. RT_INV_BALLOT: as the mask itself (inverse ballot: the
// SGPR mask becomes the branch's exec / vcc mask, no per-lane shift and compare on the VALU)
#ifndef RT_INV_BALLOT
#define RT_INV_BALLOT 0
#endif
template <bool IB = (RT_INV_BALLOT != 0)>
DEVI bool in_mask_t(uint64_t m) {
  if constexpr (IB) return __builtin_amdgcn_inverse_ballot_w64(m);
  else return (m >> __lane_id()) & 1;
}
DEVI bool in_mask(uint64_t m) { return in_mask_t<>(m); }
// MASKOPS<F>: the packet traversals' lane bits by inverse ballot and their approximate box tests as
// lane masks (slab_apx2) -- C3 3.024 -> 2.994 ms, but C4's transparent variant 453 -> 459 ms through
// its allocation, C5 unchanged (profiles/r05w_maskops_ab.log): on in the variants without
// transparent materials (RT_MASKOPS 1), everywhere (2) or nowhere (0)
#ifndef RT_MASKOPS
#define RT_MASKOPS 1
#endif
template <uint32_t F>
static constexpr bool MASKOPS = RT_MASKOPS == 2 || (RT_MASKOPS == 1 && (F & FT_TRANS) == 0);
#ifdef RT_PROF_PKSTAT
__device__ unsigned long long rt_pk_stat[16];
// one wave step testing the lanes in m: counted once per wave (by its first active lane)
#define PKSTAT(step, m)                                                                   \
  do {                                                                                    \
    const uint64_t pk_m_ = (m), pk_a_ = __ballot(1);                                      \
    if (CNT && __lane_id() == (int)__builtin_ctzll(pk_a_)) {                              \
      ct.c[step]++;                                                                       \
      ct.c[step + 1] += __builtin_popcountll(pk_m_);                                      \
    }                                                                                     \
  } while (0)
// a wave step in which some lane's condition c holds, and those lanes
#define PKSTAT_HIT(step, c)                                                               \
  do {                                                                                    \
    const uint64_t pk_h_ = __ballot(c);                                                   \
    if (pk_h_) PKSTAT(step, pk_h_);                                                       \
  } while (0)
#else
#define PKSTAT(step, m) do {} while (0)
#define PKSTAT_HIT(step, c) do {} while (0)
#endif
#ifdef RT_PROF_REGIONS
// profiling builds only (tools/regions.py): shader-clock cycles a wave spends in each region,
// accumulated per wave in LDS by its first active lane (one wave per workgroup) and added to
// the global sums once at the wave's end. Regions nest: the tool subtracts inner from outer.
enum { R_CLOSEST, R_CLOSEST_ACCEL, R_SHADOW, R_SHADOW_ACCEL, R_HIT, R_TEX, R_LIGHT, R_SHADE, R_SAMPLE, R_KERNEL,
       R_BG, R_PHOTON, R_KNN_COUNT, R_KNN_FINAL, R_KNN_NPASS, R_KNN_NCALL, R_N = 16 };
__device__ unsigned long long rt_prof_reg[R_N];
#define PROF_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(v, r)                                                                   \
  do {                                                                                   \
    const uint64_t pr_t_ = __builtin_amdgcn_s_memtime();                                 \
    if (__lane_id() == (int)__builtin_ctzll(__ballot(1))) prof_acc(r, pr_t_ - (v));      \
  } while (0)
#define PROF_CNT(r)                                                                    \
  do {                                                                                   \
    if (__lane_id() == (int)__builtin_ctzll(__ballot(1))) prof_acc(r, 1);                \
  } while (0)
#else
#define PROF_T0(v) do {} while (0)
#define PROF_ADD(v, r) do {} while (0)
#define PROF_CNT(r) do {} while (0)
#endif

DEVI double opaque_d(double x) {  // kept from being hoisted out of the traversal loop
  asm volatile("" : "+v"(x));
  return x;
}

// ---- conservative fp32 triangle pre-test (RT_F32_TRI) ------------------------------------------
// Most wave steps of the packet traversals' triangle tests have no lane that hits (C3: 83 % of the
// nearest-first closest-hit steps, 82 % of the shadow steps; profiles/r06v_pkstat_c3.json), yet each
// runs the fp64 test with its IEEE division (planar_test; myPlanarObject.java:165-211). A lane is
// first tested in fp32 against the triangle's edges, without the division, and counted out only when
// that is certain; a wave whose lanes are all out skips the fp64 test. The reference's edge value at
// its hit point is, in real arithmetic, g_j = (p - v_j) x e_j . n with p = o + t d, t = -(n.o + dA) / s,
// s = n.d (the same for both vertex orders of Q5), and it rejects when g_j < -EPS. Scaled by |s|:
//   G_j = g_j |s| = |s| (o.m_j - c_j) - sign(s) (n.o + dA) (d.m_j),  m_j = e_j x n,  c_j = v_j.m_j,
// a polynomial in the fp32-rounded inputs. Its fp32 value is within 28 u |m_j| max(1,|n|) |d| (|o| + tm)
// of the real one (u = 2^-24: input roundings plus the fma chain), the reference's own fp64 value of
// g_j |s| within ~2^-50 of the same scale; TriF.k = 2^-17 |m|max max(1,|n|) covers both with a 4x
// margin (|o|, |d| taken as 1-norms >= the 2-norms), 2^-40 |d| the fp32 rounding of EPS |s|, 2^-100
// the flushed denormals. So G'_j < -(EPS |s'| + B) implies g_j < -EPS: the reference's test fails on
// that edge whatever its t -- the lane's result is false, which is all the pre-test ever decides.
// It decides nothing where s' is within its rounding of 0 (the sign of s could differ) or B is large
// enough for a product to overflow; a non-finite record has k = +inf (B = +inf or NaN: no compare holds).
#ifndef RT_F32_TRI
#define RT_F32_TRI 1
#endif
#ifndef RT_F32_TRI_CPK  // ... in the reference-order closest hit (leaf_closest) too
#define RT_F32_TRI_CPK 1
#endif
// Measured (same-box A/Bs, same image hashes): C3 2.867 -> 2.824 ms (nearest-first closest hit + shadow
// rays), C4 489 -> 465 ms (+ the reference-order closest hit: 489 without it); the photon-map variant
// loses with it in either traversal (C5 173.0 ms without, 175.6 / 175.1 ms with it in the closest hit /
// both), so it is off there (profiles/r06w_*, r06y_f32_tri_ab.log, r06z_f32_tri_photon_ab.log)
#ifndef RT_F32_TRI_PH_ANY  // ... in the photon-map variant's shadow rays
#define RT_F32_TRI_PH_ANY 0
#endif
#ifndef RT_F32_TRI_PH_CPK  // ... in the photon-map variant's closest hit
#define RT_F32_TRI_PH_CPK 0
#endif
struct TriRayF {
  float o[3], d[3];
  float O, D;  // |o'|_1, |d'|_1
};
DEVI TriRayF tri_ray_f32(V o, V d) {  // opaque: built per leaf, not hoisted and held through the traversal
  TriRayF r;
  r.o[0] = (float)opaque_d(o.x); r.o[1] = (float)opaque_d(o.y); r.o[2] = (float)opaque_d(o.z);
  r.d[0] = (float)opaque_d(d.x); r.d[1] = (float)opaque_d(d.y); r.d[2] = (float)opaque_d(d.z);
  r.O = fabsf(r.o[0]) + fabsf(r.o[1]) + fabsf(r.o[2]);
  r.D = fabsf(r.d[0]) + fabsf(r.d[1]) + fabsf(r.d[2]);
  return r;
}
struct TriFR {  // a TriF, scalar-loaded
  float m[9], c[3], n[3], d, k, tm;
};
DEVI TriFR sload_trif(const TriF* p) {
  TriFR t;
#pragma unroll
  for (int i = 0; i < 9; ++i) t.m[i] = sload(&p->m[0][0] + i);
#pragma unroll
  for (int i = 0; i < 3; ++i) { t.c[i] = sload(p->c + i); t.n[i] = sload(p->n + i); }
  t.d = sload(&p->d); t.k = sload(&p->k); t.tm = sload(&p->tm);
  return t;
}
static constexpr float EPS_F32_UP = 1.00000001168609742e-07f;  // RN(1e-7) >= EPS
// true: the reference's triangle test certainly returns false for this lane
DEVI bool tri_f32_out(const TriFR& T, const TriRayF& r) {
  const float s = __builtin_fmaf(T.n[2], r.d[2], __builtin_fmaf(T.n[1], r.d[1], T.n[0] * r.d[0]));
  const float P = __builtin_fmaf(T.n[2], r.o[2], __builtin_fmaf(T.n[1], r.o[1], __builtin_fmaf(T.n[0], r.o[0], T.d)));
  const float as = fabsf(s), sP = s < 0 ? -P : P;
  const float B = __builtin_fmaf(r.D, __builtin_fmaf(T.k, r.O + T.tm, 0x1p-40f), 0x1p-100f);
  const float thr = -__builtin_fmaf(EPS_F32_UP, as, B);
  bool out = false;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float* m = T.m + 3 * j;
    const float Q = __builtin_fmaf(m[2], r.o[2], __builtin_fmaf(m[1], r.o[1], __builtin_fmaf(m[0], r.o[0], -T.c[j])));
    const float R = __builtin_fmaf(m[2], r.d[2], __builtin_fmaf(m[1], r.d[1], m[0] * r.d[0]));
    out = out || (__builtin_fmaf(as, Q, -(sP * R)) < thr);
  }
  return out && as > 0x1p-20f * r.D && B < 0x1p100f;
}

// a primitive test whose triangle record is loaded at a wave-uniform address (PK)
template <bool CNT, uint32_t F, bool PK, class LIM = LimNone>
DEVI bool test_ref_u(const SceneD& S, int32_t ref, V o, V d, const Key& k, double& t, int& args, Counters& ct,
                     const LIM& lim = LIM()) {
  if constexpr (PK) {
    if (!(F & FT_PRIM) || ref >= 0) {
      if (CNT) ct.c[C_TRI]++;
      WCNT(C_WTRI, 1);
      const TriG T = sload_tri(S.tri + ref);
      return tri_test(T, o, d, t, args, lim);
    }
  }
  return test_ref<CNT, F, LIM, PK>(S, ref, o, d, k, t, args, ct, lim);
}
template <uint32_t F, bool PK>
DEVI int32_t ref_xf_u(const SceneD& S, int32_t ref) {
  if (PK && (!(F & FT_PRIM) || ref >= 0)) return sload(&S.tri[ref].xf);
  return ref_xf<F>(S, ref);
}
template <uint32_t F>
DEVI bool is_inst(const SceneD& S, int32_t ref) { return (F & FT_INST) && ref < 0 && S.prim[~ref].type == PT_INST; }

// The reference returns a best hit per BVH node and merges children keeping the first of
// equal t (TreeMap); over the whole scan that is "the first-visited hit of minimal t", so
// one running best with strict-< replacement in visit order gives the same answer. What
// the per-node results are still needed for is the pruning rule (below), which only
// needs each subtree's minimal t -- a double per stack frame.

// a leaf from its child code c = ~ref (rt_types.h): a LeafD or a packed triangle run
struct LeafR {
  int32_t start, count;
  bool run;
};
template <bool PK = false>
DEVI LeafR leaf_of(const SceneD& S, int32_t c) {
  LeafR r;
  r.run = (c & LEAF_RUN_FLAG) != 0;
  if (r.run) { r.start = (c >> 5) & LEAF_RUN_MAXSTART; r.count = c & 31; }
  else if (PK) { r.start = sload(&S.leaf[c].start); r.count = sload(&S.leaf[c].count); }
  else { LeafD lf = S.leaf[c]; r.start = lf.start; r.count = lf.count; }
  return r;
}
template <bool PK = false>
DEVI int32_t leaf_member(const SceneD& S, const LeafR& lf, int i) {
  return lf.run ? lf.start + i : (PK ? sload(S.member + lf.start + i) : S.member[lf.start + i]);
}

template <bool CNT, uint32_t F>
DEVI void inst_closest(const SceneD& S, int32_t ii, WRay& w, const Key& k, int top, Best& best, double& local, Counters& ct);

// myGeomList.traverseStruct leaf loop (myGeomBase.java:281-296): strict <, leaf order.
// w is the leaf's `_ray`: the world ray, or (INST) the instance ray of an instanced accel;
// accXf >= 0: members with that CTM reuse the accel-space ray (ao, ad) while w is unchanged.
// PK: `leaf` is wave-uniform (packet traversal): member records are loaded as scalars.
template <bool CNT, uint32_t F, bool INST, bool PK = false>
DEVI void leaf_closest(const SceneD& S, int32_t leaf, int accXf, V ao, V ad, WRay& w, const Key& k, const HitCtx& hc,
                       Best& best, double& local, Counters& ct) {
  const LeafR lf = leaf_of<PK>(S, leaf);
  if (CNT) { ct.c[C_LEAF]++; ct.c[C_MEMBER] += lf.count; }
  // the fp32 triangle pre-test (members in the accel's CTM; RT_F32_TRI_CPK)
  constexpr bool TF32 = PK && !INST && RT_F32_TRI != 0 && RT_F32_TRI_CPK != 0 &&
                        ((F & FT_PHOTON) == 0 || RT_F32_TRI_PH_CPK != 0);
  TriRayF trf;
  if constexpr (TF32) trf = tri_ray_f32(ao, ad);
  for (int i = 0; i < lf.count; ++i) {
    if (PK) PKSTAT(P_CT_STEP, __ballot(1));
    int32_t ref = leaf_member<PK>(S, lf, i);
    renorm(w);  // _ray.getTransformedRay(_ray, obj.CTMara[invIDX])
    if constexpr (!INST && (F & FT_INST) != 0) {
      if (is_inst<F>(S, ref)) {  // a sierpinski element: myInstance.intersectCheck
        inst_closest<CNT, F>(S, ~ref, w, k, hc.top, best, local, ct);
        continue;
      }
    }
    int xf = ref_xf_u<F, PK>(S, ref);
    V o, d;
    if (xf == accXf && !w.moved) { o = ao; d = ad; }
    else if (PK && (RT_ULOAD & 1)) {  // xf is wave-uniform here (ref_xf_u): the inverse as scalar loads
      double inv[12];
      sload_inv(S.xf + xf, inv);
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    } else { const double* inv = S.xf[xf].inv; o = xpt(inv, w.o); d = xvec(inv, w.d); }
    double t;
    int args;
    bool th;
    if (TF32 && (!(F & FT_PRIM) || ref >= 0) && xf == accXf && !w.moved) {  // test_ref_u's triangle case
      if (CNT) ct.c[C_TRI]++;
      WCNT(C_WTRI, 1);
      const TriFR TF = sload_trif(S.triF + ref);
      th = false;
      if (!tri_f32_out(TF, trf)) {
        const TriG T = sload_tri(S.tri + ref);
        th = tri_test(T, o, d, t, args, LimClosest{local, best.t});
      }
    } else {
      th = test_ref_u<CNT, F, PK>(S, ref, o, d, k, t, args, ct, LimClosest{local, best.t});
    }
    if (th) {
      if (t < local) local = t;
      if (t < best.t) {
        best.t = t; best.ref = ref; best.top = (int16_t)hc.top; best.inAcc = 1; best.inst = hc.inst;
        if (INST) { best.ver = hc.wver; best.iver = w.ver; }
        else { best.ver = w.ver; best.iver = 0; }
      }
    }
  }
}

static constexpr int BVH_STACK = 40;  // host rejects BVHs deeper than 40

// Traversal stacks: the first NL levels live in LDS ([level][lane], conflict-free),
// deeper levels in scratch. The closest-hit and shadow traversals never overlap in time,
// so they share the LDS node-index array. One wave per workgroup. The traversal of an
// instanced accel runs while the enclosing one is suspended: it keeps its whole stack in
// scratch (NL = 0).
#ifndef RT_STACK_LDS
#define RT_STACK_LDS 12
#endif
static constexpr int STK_LDS = RT_STACK_LDS;
// dynamic LDS of every kernel here: the traversal stack, aliased by render_kernel's
// per-round sample colours (used only between traversals)
extern __shared__ double rt_lds[];
static constexpr int LDS_STACK_BYTES = STK_LDS * 64 * 12;
// Packet traversal (below): per-lane subtree minima for the first PK_LDS levels
// ([level][lane] doubles), then the wave-uniform frames: lane masks (subtree; right box
// hit, shadow rays), node<<1|phase and the right child (shadow rays).
#ifndef RT_PK_LDS
#define RT_PK_LDS 16
#endif
static constexpr int PK_LDS = RT_PK_LDS;
static constexpr int PKO_M = PK_LDS * 64 * 8;  // byte offsets in rt_lds
static constexpr int PKO_R = PKO_M + BVH_STACK * 8;
static constexpr int PKO_N = PKO_R + BVH_STACK * 8;
static constexpr int PKO_C = PKO_N + BVH_STACK * 4;
static constexpr int LDS_PK_BYTES = PKO_C + BVH_STACK * 4;
static constexpr int LDS_MAX2 = LDS_STACK_BYTES > LDS_PK_BYTES ? LDS_STACK_BYTES : LDS_PK_BYTES;
static constexpr int LDS_BASE_BYTES = LDS_MAX2 > 64 * 4 * 8 ? LDS_MAX2 : 64 * 4 * 8;
#ifdef RT_PROF_REGIONS
static constexpr int LDS_BYTES = LDS_BASE_BYTES + R_N * 8;  // + the wave's region accumulators
#else
static constexpr int LDS_BYTES = LDS_BASE_BYTES;
#endif
// render kernel: + the per-pixel colour sums of a multi-round sample loop (G >= 2: at most 32
// pixels per wave), kept in LDS across the shading trees instead of in VGPRs
static constexpr int SUM_BYTES = 32 * 3 * 8;
// + the lane masks of one group of lights whose shadow rays are traced compacted (light_sum_w)
static constexpr int GRP_MAX = 8;
static constexpr int GRP_BYTES = GRP_MAX * 8;
static constexpr int LDS_RENDER_BYTES = LDS_BYTES + SUM_BYTES + GRP_BYTES;
static_assert(16 * LDS_RENDER_BYTES <= 160 * 1024, "16 waves per CU");
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) int32_t lds_i32;
DEVI lds_f64* ldsT() { return (lds_f64*)rt_lds; }
DEVI lds_i32* ldsN() { return (lds_i32*)(rt_lds + STK_LDS * 64); }
template <int NL>
struct StackT {
  double sT[BVH_STACK - NL];
  int32_t sN[BVH_STACK - NL];
  DEVI double getT(int i) const {
    if (NL > 0 && i < NL) return ldsT()[i * 64 + threadIdx.x];
    return sT[i - NL];
  }
  DEVI void setT(int i, double v) {
    if (NL > 0 && i < NL) ldsT()[i * 64 + threadIdx.x] = v;
    else sT[i - NL] = v;
  }
  DEVI int32_t getN(int i) const {
    if (NL > 0 && i < NL) return ldsN()[i * 64 + threadIdx.x];
    return sN[i - NL];
  }
  DEVI void setN(int i, int32_t v) {
    if (NL > 0 && i < NL) ldsN()[i * 64 + threadIdx.x] = v;
    else sN[i - NL] = v;
  }
};
typedef StackT<STK_LDS> Stack;

template <int NL>
struct NStackT {  // shadow traversal: node indices only
  int32_t sN[BVH_STACK - NL];
  DEVI int32_t getN(int i) const {
    if (NL > 0 && i < NL) return ldsN()[i * 64 + threadIdx.x];
    return sN[i - NL];
  }
  DEVI void setN(int i, int32_t v) {
    if (NL > 0 && i < NL) ldsN()[i * 64 + threadIdx.x] = v;
    else sN[i - NL] = v;
  }
};
typedef NStackT<STK_LDS> NStack;

// myAccelStruct.intersectCheck + myBVH.traverseStruct (myGeomBase.java:216-222, 407-421),
// iteratively with the reference's LOCAL pruning: the right child is visited iff its
// box is hit and (left subtree missed or box entry t < the LEFT SUBTREE's minimal t);
// ties go left. A frame = the enclosing subtree's minimal t so far + node<<1|phase; the
// right box is tested when the left subtree is done, as the Java does.
// INST: an instanced accel, whose `_ray` and `_trans` are the same ray object: the boxes
// are tested with w itself, re-normalised in place by the leaves (myInstance.intersectCheck).
template <bool CNT, uint32_t F, bool INST>
DEVI void accel_closest(const SceneD& S, const AccelD& A, V ao, V ad, RayInv ri, WRay& w, const Key& k,
                        const HitCtx& hc, Best& best, double& outer, Counters& ct) {
  StackT<INST ? 0 : STK_LDS> st;
  int sp = 0;
  double local = DMAX;
  int32_t N = A.root;  // a leaf root (a plain list) is tested by the same loop with no frames
  while (true) {
    // descend: push N, go left while the left box is hit
    while (N >= 0) {
      const NodeD& nd = S.node[N];
      if (CNT) { ct.c[C_NODE]++; ct.c[C_WNODE]++; ct.c[C_BOX] += 2; }  // both child boxes are tested once per visit
      st.setT(sp, local);
      st.setN(sp, N << 1);
      sp++;
      local = DMAX;
      if (box_hit<MASKOPS<F>>(nd.lmin, nd.lmax, ao, ad, ri)) N = nd.left;
      else { N = INT32_MAX; break; }
    }
    if (N != INT32_MAX) {
      leaf_closest<CNT, F, INST>(S, ~N, INST ? -1 : A.xf, ao, ad, w, k, hc, best, local, ct);
      if (INST && w.moved) { ad = w.d; ri = ray_inv(ao, ad, S.fastSlab & SCENE_FAST_SLAB); w.moved = false; }
    }
    // unwind
    N = INT32_MAX;
    while (sp > 0) {
      const int32_t np = st.getN(sp - 1);
      if ((np & 1) == 0) {
        const NodeD& nd = S.node[np >> 1];
        if (box_before<MASKOPS<F>>(nd.rmin, nd.rmax, ao, ad, ri, local)) {
          st.setN(sp - 1, np | 1);
          N = nd.right;
          break;
        }
      }
      // this node's minimal t joins the enclosing subtree's
      const double sv = st.getT(sp - 1);
      if (sv < local) local = sv;
      sp--;
    }
    if (N == INT32_MAX) break;
  }
  if (local < outer) outer = local;
}

// ---------------------------------------------------------------------------
// Packet traversal. The lanes of a wave trace nearly the same rays (the samples of a
// 2x2 pixel tile), so the wave walks ONE node sequence -- the union of its lanes' --
// with wave-uniform control: node indices, frames and lane masks live in SGPRs / LDS,
// node and triangle records are scalar loads (s_load into SGPRs), and a lane executes
// the box and leaf tests only at the nodes its own sequential traversal visits (lane
// mask per frame). Each lane therefore performs exactly the tests of accel_closest /
// accel_any above, in the same order, with the same pruning -- the results (and the
// instrumented counters) are identical; only idle lanes wait.
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) char lds_u8;
DEVI lds_u8* pkB() { return (lds_u8*)rt_lds; }
DEVI lds_f64* pkT() { return (lds_f64*)rt_lds; }
DEVI lds_u64* pkM() { return (lds_u64*)(pkB() + PKO_M); }
// Per-lane LDS spill slots for the shading of a hit (shade_node / light_sum, packet kernels):
// while a hit is shaded, the closest-hit traversal's per-lane subtree-minimum levels (pkT)
// and the sample-colour buffer are idle -- shadow rays and the photon gather use only the
// wave-uniform frames -- so the values that must outlive every shadow-ray scan (normal, view
// direction, texture colour, the light sums) wait there instead of in VGPRs, and the scan's
// traversal keeps its ray in registers. A compiler barrier after the stores makes every later
// read come from LDS.
// slots: while light_sum runs -- the node's ambient (+ photon) colour, ltMult, texture colour,
// normal, view direction, light sums; between two rays of a shading tree -- the next ray.
// With compacted shadow rays (light_sum_w) the light sums stay in registers and slots 3 / 13..15
// hold the hit's RNG key and point, which the lanes tracing its shadow rays read.
enum { SL_BASE = 0, SL_LTM = 3, SL_TEX = 4, SL_NRM = 7, SL_DW = 10, SL_RGB = 13, SL_N = 16, SL_RAYO = 0, SL_RAYD = 3,
       SL_KEY = 3, SL_FWD = 13 };
DEVI void stash(int q, double v) { pkT()[q * 64 + __lane_id()] = v; }
// A wave-uniform value (kernel argument, in SGPRs) made opaque where it is used: what is derived
// from it (its copy into VGPRs, a conversion) is then computed at the use instead of being hoisted
// out of the sample loop and spilled to scratch across the shading tree -- a per-wave store of 64
// copies of the same value (RT_UNI_OPAQUE; C3 wrote ~4 KB per wave that way at the loop's entry)
#ifndef RT_UNI_OPAQUE
#define RT_UNI_OPAQUE 1
#endif
template <class T>
DEVI T uni_here(T v) {
  if (RT_UNI_OPAQUE) asm volatile("" : "+s"(v));
  return v;
}
DEVI double unstash(int q) { return pkT()[q * 64 + __lane_id()]; }
DEVI void stash3(int q, V v) { stash(q, v.x); stash(q + 1, v.y); stash(q + 2, v.z); }
DEVI V unstash3(int q) { return mk(unstash(q), unstash(q + 1), unstash(q + 2)); }
DEVI void lds_barrier() { asm volatile("" ::: "memory"); }
#ifdef RT_PROF_REGIONS
DEVI lds_u64* profL() { return (lds_u64*)(pkB() + LDS_BASE_BYTES); }
DEVI void prof_acc(int r, uint64_t dt) { profL()[r] += dt; }
#endif
DEVI lds_u64* pkR() { return (lds_u64*)(pkB() + PKO_R); }
DEVI lds_i32* pkN() { return (lds_i32*)(pkB() + PKO_N); }
DEVI lds_i32* pkC() { return (lds_i32*)(pkB() + PKO_C); }
struct PkStack {
  double sT[BVH_STACK - PK_LDS];  // per-lane subtree minima below the LDS levels
  DEVI double getT(int i) const { return i < PK_LDS ? pkT()[i * 64 + __lane_id()] : sT[i - PK_LDS]; }
  DEVI void setT(int i, double v) {
    if (i < PK_LDS) pkT()[i * 64 + __lane_id()] = v;
    else sT[i - PK_LDS] = v;
  }
  // wave-uniform frame: every active lane writes the same value; read back as a scalar
  DEVI void setFrame(int i, int32_t n, uint64_t m) { pkN()[i] = n; pkM()[i] = m; }
  DEVI void setN(int i, int32_t n) { pkN()[i] = n; }
  DEVI int32_t getN(int i) const { return uni(pkN()[i]); }
  DEVI uint64_t getM(int i) const { return uni64(pkM()[i]); }
  // shadow frames: + the lanes whose right-child box is hit (tested at the push) and the right child
  DEVI void setFrameR(int i, int32_t n, uint64_t m, uint64_t r, int32_t c) {
    pkN()[i] = n; pkM()[i] = m; pkR()[i] = r; pkC()[i] = c;
  }
  DEVI uint64_t getR(int i) const { return uni64(pkR()[i]); }
  DEVI int32_t getC(int i) const { return uni(pkC()[i]); }
};

// ---- conservative fp32 box pre-test (RT_F32_BOX) ---------------------------------------------
// The packet traversals' child-box tests first run in fp32 on the node's fp32 boxes (NodeF): a
// wave64 f32 fma / add / min is issued at twice the rate of its fp64 form on gfx950, and the whole
// test is ~22 instructions instead of ~30 fp64 ones (tools/valu_issue.hip). A decision
// is taken from fp32 only when it is certain, and then it is the reference's (myBBox.intersectCheck,
// myGeomBase.java:132-162); every other lane runs the existing fp64 tests. The bound: with
// t = (b - o) y (real, y the fp64 reciprocal), the fp32 slab value t' = fma(RN(b), RN(y), RN(-RN(o) RN(y)))
// satisfies |t' - t| <= 2^-21 |y| (|b| + |o|) (four roundings of 2^-24, |t| <= |y| (|b| + |o|)), so with
// E = 2^-20 ymax (mag + omax) (mag >= |b| over the node's two boxes, both bounds rounded up) the fp32
// entry / exit lo', hi' are within E of the real ones, and each fp32 compare below rounds by at most
// 2^-24 of values <= 2^20 E: a miss is certain when hi' < lo' - 4E or lo' < -2E, a hit when
// hi' > lo' + 4E and lo' > 2E (the reference's own rounding, ~2^-51 relative, is far inside these
// margins). Overflow makes E (and the test) +inf or NaN: nothing is settled then.
#ifndef RT_F32_BOX
#define RT_F32_BOX 1
#endif
// In the shadow (any-hit) packet traversal: C4 482 -> 453 ms, C5 175.1 -> 173.4 ms; in C3's
// triangles-only variant only with the fp32 ray rebuilt per node from the fp64 one (RT_F32_SH_LAZY:
// held through the traversal its registers made the shading code spill, 2.90 -> 2.96 ms; rebuilt,
// 2.90 -> 2.87 ms, and C4 453 -> 450 ms; the photon variant keeps it held, C5 173.3 vs 174.6 ms).
// The nearest-first closest hit gains in C3 (2.94 -> 2.90 ms). Same images (profiles/r06f_f32_ab.log,
// r06h_f32_ab_same_box.log, r06j_f32_lazy_ab.log).
#ifndef RT_F32_SHADOW  // the fp32 pre-test in the shadow (any-hit) packet traversal
#define RT_F32_SHADOW 1
#endif
#ifndef RT_F32_SHADOW_TRANS  // ... of the transparent variants
#define RT_F32_SHADOW_TRANS 1
#endif
#ifndef RT_F32_SHADOW_OPAQUE  // ... of the other variants (with the fp32 ray rebuilt per node, RT_F32_SH_LAZY)
#define RT_F32_SHADOW_OPAQUE 1
#endif
struct RayF {
  float y[3], noy[3];  // RN(y_i), RN(-RN(o_i) RN(y_i))
  float ymax, omax;    // >= max |y_i|, >= max |o_i|
};
DEVI RayF ray_f32(V o, const RayInv& ri, double ymax) {
  RayF r;
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  r.y[0] = (float)ri.y[0]; r.y[1] = (float)ri.y[1]; r.y[2] = (float)ri.y[2];
  r.noy[0] = -(ox * r.y[0]); r.noy[1] = -(oy * r.y[1]); r.noy[2] = -(oz * r.y[2]);
  r.ymax = (float)(ymax * (1 + 0x1p-20));
  r.omax = (float)(fmax(fmax(fabs(o.x), fabs(o.y)), fabs(o.z)) * (1 + 0x1p-20));
  return r;
}
// the per-axis part of ray_f32 alone (RT_F32_SH_LAZY)
DEVI RayF ray_f32_dirs(V o, const RayInv& ri) {
  RayF r;
  const float ox = (float)opaque_d(o.x), oy = (float)opaque_d(o.y), oz = (float)opaque_d(o.z);
  r.y[0] = (float)opaque_d(ri.y[0]); r.y[1] = (float)opaque_d(ri.y[1]); r.y[2] = (float)opaque_d(ri.y[2]);
  r.noy[0] = -(ox * r.y[0]); r.noy[1] = -(oy * r.y[1]); r.noy[2] = -(oz * r.y[2]);
  r.ymax = r.omax = 0;
  return r;
}
// The same pre-test in the reference-order closest hit of the transparent variants (RT_F32_CPK) does
// not pay: C4 450.8 -> 451.9 ms, C5 173.1 -> 175.8 ms (profiles/r06n_f32_cpk_ab.log) -- those
// traversals test one box per step and the fp64 box's SGPRs were already loaded; off.
#ifndef RT_F32_CPK  // the fp32 pre-test in the reference-order closest hit of the transparent variants
#define RT_F32_CPK 0
#endif
#ifndef RT_F32_CPK_PHOTON  // ... of the photon-map variant too
#define RT_F32_CPK_PHOTON 1
#endif
#ifndef RT_F32_SH_LAZY  // (variants without a photon map)
#define RT_F32_SH_LAZY 1
#endif
DEVI float f32_margin(const RayF& r, float mag) { return 0x1p-20f * (r.ymax * (mag + r.omax)); }
enum : int { B32_MISS = 0, B32_HIT = 1, B32_OPEN = 2 };
// b: min[3] max[3] of one child (fp32); lo: the fp32 entry (a settled hit's entry within E)
DEVI int box32(const float* b, const RayF& r, float E, float& lo) {
  const float t0 = __builtin_fmaf(b[0], r.y[0], r.noy[0]), t3 = __builtin_fmaf(b[3], r.y[0], r.noy[0]);
  const float t1 = __builtin_fmaf(b[1], r.y[1], r.noy[1]), t4 = __builtin_fmaf(b[4], r.y[1], r.noy[1]);
  const float t2 = __builtin_fmaf(b[2], r.y[2], r.noy[2]), t5 = __builtin_fmaf(b[5], r.y[2], r.noy[2]);
  lo = fmaxf(fmaxf(fminf(t0, t3), fminf(t1, t4)), fminf(t2, t5));
  const float hi = fminf(fminf(fmaxf(t0, t3), fmaxf(t1, t4)), fmaxf(t2, t5));
  if (hi < lo - 4 * E || lo < -2 * E) return B32_MISS;
  if (hi > lo + 4 * E && lo > 2 * E) return B32_HIT;
  return B32_OPEN;
}
// nf_child's lower bound of a settled hit's grown entry: lo_real - s ymax >= (lo' - E) - s ymax, and
// the two fp32 roundings here are covered by the further 2E and by s, ymax being rounded up
DEVI double lb32(float lo, float E, float s, const RayF& r) { return (double)((lo - 3 * E) - s * r.ymax); }
struct NodeBoxF {  // a node's fp32 record, scalar-loaded
  float b[12];
  float mag, sl, sr;
};
DEVI NodeBoxF sload_nodef(const NodeF* p) {
  NodeBoxF n;
#pragma unroll
  for (int i = 0; i < 12; ++i) n.b[i] = sload(p->b + i);
  n.mag = sload(&p->mag); n.sl = sload(&p->sl); n.sr = sload(&p->sr);
  return n;
}
DEVI int32_t sload_ref(const NodeD* nd, int side) { return sload(side ? &nd->right : &nd->left); }


// accel_closest<INST = false> as a packet traversal (same per-lane semantics)
template <bool CNT, uint32_t F>
DEVI void accel_closest_pk(const SceneD& S, const AccelD& A, V ao, V ad, RayInv ri, WRay& w, const Key& k,
                           const HitCtx& hc, Best& best, double& outer, Counters& ct) {
  PkStack st;
  int sp = 0;
  double local = DMAX;
  uint64_t act = __ballot(1);  // lanes in the current subtree
  int32_t N = uni(A.root);
  const int32_t axf = A.xf;
  // the fp32 box pre-test (box32) in the transparent variants, whose closest hit takes this
  // reference-order traversal (not C3's, where it is only the fat-edge fallback)
  constexpr bool F32 = RT_F32_BOX && RT_F32_CPK && (F & FT_TRANS) != 0 && (RT_F32_CPK_PHOTON || (F & FT_PHOTON) == 0);
  constexpr bool LAZY = RT_F32_SH_LAZY != 0 && (F & FT_PHOTON) == 0;
  const bool f32 = F32 && ri.fast;
  RayF rf;
  if constexpr (F32) rf = ray_f32(ao, ri, fmax(fmax(fabs(ri.y[0]), fabs(ri.y[1])), fabs(ri.y[2])));
  auto rebuild = [&]() {
    if constexpr (F32 && LAZY) {
      const RayF r2 = ray_f32_dirs(ao, ri);
      rf.y[0] = r2.y[0]; rf.y[1] = r2.y[1]; rf.y[2] = r2.y[2];
      rf.noy[0] = r2.noy[0]; rf.noy[1] = r2.noy[1]; rf.noy[2] = r2.noy[2];
    }
  };
  while (true) {
    // descend: push N, go left with the lanes whose left box is hit
    while (N >= 0) {
      st.setFrame(sp, N << 1, act);
      PKSTAT(P_CB_STEP, act);
      WCNT(C_WNODE, 1);  // the node's record: left half now, right half at the unwind
      bool hl = false;
      int32_t lref;
      if constexpr (F32) {
        const NodeD* nd = S.node + N;
        lref = sload_ref(nd, 0);
        bool open = false;
        if (in_mask_t<MASKOPS<F>>(act)) {
          if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX] += 2; }
          st.setT(sp, local);
          local = DMAX;
          if (f32) {
            rebuild();
            float b[6], mag;
#pragma unroll
            for (int i = 0; i < 6; ++i) b[i] = sload(S.nodeF[N].b + i);
            mag = sload(&S.nodeF[N].mag);
            float lo;
            const int c = box32(b, rf, f32_margin(rf, mag), lo);
            hl = c == B32_HIT;
            open = c == B32_OPEN;
          } else {
            open = true;
          }
        }
        if (__ballot(open)) {
          const ChildBox cl = sload_child(nd, 0);
          if (open) hl = box_hit<MASKOPS<F>>(cl.mn, cl.mx, ao, ad, ri);
        }
      } else {
        const ChildBox cl = sload_child(S.node + N, 0);
        lref = cl.ref;
        if (in_mask_t<MASKOPS<F>>(act)) {
          if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX] += 2; }
          st.setT(sp, local);
          local = DMAX;
          hl = box_hit<MASKOPS<F>>(cl.mn, cl.mx, ao, ad, ri);
        }
      }
      sp++;
      const uint64_t H = __ballot(hl);
      if (H) { act = H; N = lref; }
      else { N = INT32_MAX; break; }
    }
    if (N != INT32_MAX && in_mask_t<MASKOPS<F>>(act)) leaf_closest<CNT, F, false, true>(S, ~N, axf, ao, ad, w, k, hc, best, local, ct);
    // unwind
    N = INT32_MAX;
    while (sp > 0) {
      const int32_t np = st.getN(sp - 1);
      const uint64_t M = st.getM(sp - 1);
      if ((np & 1) == 0) {
        PKSTAT(P_CB_STEP, M);
        bool gr = false;
        int32_t rref;
        if constexpr (F32) {
          // hit and (local == DMAX or entry < local): settled when the entry is clear of local
          const NodeD* nd = S.node + (np >> 1);
          rref = sload_ref(nd, 1);
          bool open = false;
          if (in_mask_t<MASKOPS<F>>(M)) {
            if (f32) {
              rebuild();
              float b[6], mag;
#pragma unroll
              for (int i = 0; i < 6; ++i) b[i] = sload(S.nodeF[np >> 1].b + 6 + i);
              mag = sload(&S.nodeF[np >> 1].mag);
              float lo;
              const float E = f32_margin(rf, mag);
              const int c = box32(b, rf, E, lo);
              if (c == B32_HIT) {
                const double lt = fabs(local) * 0x1p-40;
                if (local == DMAX || (double)(lo + 2 * E) < local - lt) gr = true;
                else if (!((double)(lo - 2 * E) > local + lt)) open = true;
              } else {
                open = c == B32_OPEN;
              }
            } else {
              open = true;
            }
          }
          if (__ballot(open)) {
            const ChildBox cr = sload_child(nd, 1);
            if (open) gr = box_before<MASKOPS<F>>(cr.mn, cr.mx, ao, ad, ri, local);
          }
        } else {
          const ChildBox cr = sload_child(S.node + (np >> 1), 1);
          rref = cr.ref;
          if (in_mask_t<MASKOPS<F>>(M)) gr = box_before<MASKOPS<F>>(cr.mn, cr.mx, ao, ad, ri, local);
        }
        const uint64_t R = __ballot(gr);
        if (R) {
          st.setN(sp - 1, np | 1);
          act = R;
          N = rref;
          break;
        }
      }
      // this node's minimal t joins the enclosing subtree's
      if (in_mask_t<MASKOPS<F>>(M)) {
        const double sv = st.getT(sp - 1);
        if (sv < local) local = sv;
      }
      act = M;
      sp--;
    }
    if (N == INT32_MAX) break;
  }
  if (local < outer) outer = local;
}

// ---------------------------------------------------------------------------
// Nearest-first closest hit (packet), for BVHs of triangle runs in the accel's own CTM
// (AccelD.flags ACCEL_NEAREST) and rays the in-place re-normalisation no longer changes.
//
// The reference visits a BVH left child first and prunes only a RIGHT child, against its left
// sibling's subtree minimum (accel_closest). Its answer is nevertheless a function of the hits
// alone: call h* the hit of minimal t over every leaf the reference's box tests reach (Q2 boxes:
// origin inside = miss), ties to the first in depth-first leaf order -- the triangle index, as
// pack_leaves numbers triangles in leaf order. If h*'s point lies inside its leaf's box (so the
// ray enters every box above it before t*), the reference returns h*: it visits every left child
// whose box is hit, and a right child R above h* is pruned only if the left sibling's subtree
// holds a hit with t <= entry(R) < t*, which would beat or precede h*. This traversal finds h*
// with the smallest work: children nearest first, a child skipped when the ray enters its box
// grown by the fat-edge bound (node_slack: every point the triangle test accepts below it lies
// within) beyond the best hit so far -- such a subtree holds no hit that could win or tie. The
// reference's exact box test still decides reachability. A lane whose winner lies outside its
// leaf box (a fat-edge hit) re-runs the reference traversal (accel_closest_pk). The image is the
// reference's bit for bit; the counting kernel under RT_RENDER_NOCULL keeps the reference order,
// so its counters remain the reference algorithm's.
#ifndef RT_NEAREST_FIRST
#define RT_NEAREST_FIRST 1
#endif
// The child being entered is kept as a code (node << 1 | side) and its box reloaded (scalar loads) only
// when a lane finds a new best hit in the leaf, instead of the 13-SGPR box riding along the whole
// traversal: at the SGPR limit it was being moved to VGPRs and spilled (C3: 3.22 -> 3.05 ms per frame,
// scratch writes 2.30 -> 1.58 GB, reads 1.04 -> 0.67 GB; same image; profiles/r04g_*)
#ifndef RT_NF_CODE
#define RT_NF_CODE 1
#endif
#ifndef RT_NF_TRANS  // nearest-first closest hit in the transparent (non-photon) variants too
#define RT_NF_TRANS 0
#endif
#ifndef RT_AN_TRANS  // nearest-first any-hit order in the transparent variants too
#define RT_AN_TRANS 0
#endif
// (not in the photon-map and transparent variants, whose 128-VGPR allocation it perturbs: C5's
// kernel lost 10 % to the unused code, C4's 3 % -- 583 -> 599 ms -- although its bunnies use it)
static constexpr bool NEAREST_FIRST = RT_NEAREST_FIRST != 0;
DEVI double sload_slack(const NodeD* nd, int side) {
  return sload(reinterpret_cast<const double*>(side ? &nd->padR[1] : &nd->pad[1]));
}
// entry t of the box grown by s on every side (RN products with the reciprocal: within 2^-50 of
// the exact entry, far inside node_slack's 2^-30 margin); DMAX when the ray misses it
DEVI double entry_grown(const double* mn, const double* mx, double s, V o, const double* y) {
  const double t0 = ((mn[0] - s) - o.x) * y[0], t3 = ((mx[0] + s) - o.x) * y[0];
  const double t1 = ((mn[1] - s) - o.y) * y[1], t4 = ((mx[1] + s) - o.y) * y[1];
  const double t2 = ((mn[2] - s) - o.z) * y[2], t5 = ((mx[2] + s) - o.z) * y[2];
  const double lo = fmax(fmax(fmin(t0, t3), fmin(t1, t4)), fmin(t2, t5));
  const double hi = fmin(fmin(fmax(t0, t3), fmax(t1, t4)), fmax(t2, t5));
  return (hi >= lo && hi > 0) ? lo : DMAX;
}
// RT_NF_LB: a child's grown-box entry from its exact box's own slab values -- every axis's entry moves
// by at most s |y_axis| when the box grows by s, so lo - s max|y| is a lower bound of the grown entry
// within s max|y| of it: pruning by it is conservative (it prunes no subtree the exact grown entry
// keeps), ordering by it changes no answer (nearest-first finds h* in any order), and the box's hit
// decision reuses the same six slab values instead of a second slab computation. C3 2.995 -> 2.926 ms,
// same image (profiles/r05zc_c3_nf_lb_ab.log)
#ifndef RT_NF_LB
#define RT_NF_LB 1
#endif
template <bool A2>
DEVI bool nf_child(const ChildBox& c, double s, double ymax, V o, V d, const RayInv& ri, double lim, double& e) {
  if (!ri.fast) {
    e = entry_grown(c.mn, c.mx, s, o, ri.y);
    return e <= lim && box_hit<A2>(c.mn, c.mx, o, d, ri);
  }
  double lo;
  bool sure;
  const bool h = slab_apx2(c.mn, c.mx, o, ri.y, lo, sure);
  e = DMAX;
  if (sure) {  // a settled hit has a finite entry lo > 0
    if (!h) return false;
    const double lb = lo - s * ymax;  // ymax = inf (an axis-parallel ray): -inf, never pruned
    if (!(lb <= lim)) return false;
    e = lb;
    return true;
  }
  double te;  // unsettled (grazing): the exact test, and the grown entry by its own computation
  if (!slab_exact(c.mn, c.mx, o, d, ri, te)) return false;
  e = entry_grown(c.mn, c.mx, s, o, ri.y);
  return e <= lim;
}
// a candidate t worth the inside test: it can beat (or, by leaf order, tie) this accel's best
// and beats the best of the entries before it (their ties win: TreeMap keeps the first)
struct LimNF {
  double bt, prev;
  DEVI bool ok(double t) const { return t <= bt && t < prev; }
};
template <bool CNT, uint32_t F>
DEVI void accel_closest_nf(const SceneD& S, const AccelD& A, V ao, V ad, RayInv ri, WRay& w, const Key& k,
                           const HitCtx& hc, Best& best, double& outer, Counters& ct) {
  double bt = DMAX;       // this accel's best hit: t, triangle index (leaf order), point inside its leaf box
  int32_t bref = INT32_MAX;
  bool inside = false;
  uint64_t act = __ballot(1);
  int sp = 0;
  int32_t N = uni(A.root);
  const double ymax = fmax(fmax(fabs(ri.y[0]), fabs(ri.y[1])), fabs(ri.y[2]));  // RT_NF_LB
  const bool f32 = RT_F32_BOX && RT_NF_LB && RT_NF_CODE && ri.fast;
  const RayF rf = ray_f32(ao, ri, ymax);
#if RT_NF_CODE
  int32_t curCode = 0;    // the child being entered (node << 1 | side): its box is reloaded for the inside test
#else
  ChildBox cur;           // the box of the child being entered (a leaf's box when N < 0)
#endif
  while (true) {
    if (N >= 0) {  // internal: both children tested now, the nearer one entered, the other pushed
      const NodeD* nd = S.node + N;
#if RT_F32_BOX && RT_NF_LB && RT_NF_CODE
      // the fp32 pre-test on the node's 64-B fp32 record; the fp64 boxes are loaded only when a lane
      // is left unsettled (grazing rays, or a ray the pre-test cannot bound)
      const NodeBoxF nb = sload_nodef(S.nodeF + N);
      struct { int32_t ref; } cl{sload_ref(nd, 0)}, cr{sload_ref(nd, 1)};
      WCNT(C_WNODE, 1);  // a node visit (8(d) prices one at 64 B, as the reference order's)
      bool hl = false, hr = false, ol = false, orr = false;
      double el = DMAX, er = DMAX;
      const double bnd = fmin(best.t, bt), lim = fmin(bnd + bnd * 0x1p-40, 0x1p1000);  // a miss (DMAX) never passes
      if (in_mask_t<MASKOPS<F>>(act)) {
        if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX] += 2; }
        if (f32) {
          const float E = f32_margin(rf, nb.mag);
          float lo;
          const int cl32 = box32(nb.b, rf, E, lo);
          if (cl32 == B32_HIT) { el = lb32(lo, E, nb.sl, rf); hl = el <= lim; if (!hl) el = DMAX; }
          ol = cl32 == B32_OPEN;
          const int cr32 = box32(nb.b + 6, rf, E, lo);
          if (cr32 == B32_HIT) { er = lb32(lo, E, nb.sr, rf); hr = er <= lim; if (!hr) er = DMAX; }
          orr = cr32 == B32_OPEN;
        } else {
          ol = orr = true;
        }
      }
      if (__ballot(ol || orr)) {  // unsettled lanes: the fp64 tests (nf_child)
        if (__ballot(ol)) {
          const ChildBox c = sload_child(nd, 0);
          if (ol) hl = nf_child<MASKOPS<F>>(c, sload_slack(nd, 0), ymax, ao, ad, ri, lim, el);
        }
        if (__ballot(orr)) {
          const ChildBox c = sload_child(nd, 1);
          if (orr) hr = nf_child<MASKOPS<F>>(c, sload_slack(nd, 1), ymax, ao, ad, ri, lim, er);
        }
      }
#else
      const ChildBox cl = sload_child(nd, 0), cr = sload_child(nd, 1);
      const double sl = sload_slack(nd, 0), sr = sload_slack(nd, 1);
      WCNT(C_WNODE, 1);  // a node visit (8(d) prices one at 64 B, as the reference order's)
      bool hl = false, hr = false;
      double el = DMAX, er = DMAX;
      if (in_mask_t<MASKOPS<F>>(act)) {
        if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX] += 2; }
        const double bnd = fmin(best.t, bt), lim = fmin(bnd + bnd * 0x1p-40, 0x1p1000);  // a miss (DMAX) never passes
        if constexpr (RT_NF_LB != 0) {
          hl = nf_child<MASKOPS<F>>(cl, sl, ymax, ao, ad, ri, lim, el);
          hr = nf_child<MASKOPS<F>>(cr, sr, ymax, ao, ad, ri, lim, er);
        } else {
          el = entry_grown(cl.mn, cl.mx, sl, ao, ri.y);
          er = entry_grown(cr.mn, cr.mx, sr, ao, ri.y);
          if (el <= lim) hl = box_hit<MASKOPS<F>>(cl.mn, cl.mx, ao, ad, ri);
          if (er <= lim) hr = box_hit<MASKOPS<F>>(cr.mn, cr.mx, ao, ad, ri);
        }
      }
#endif
      const uint64_t L = __ballot(hl), R = __ballot(hr);
      if (L && R) {
        const int fl = (int)__builtin_ctzll(L & R);
        const bool nearLeft = __builtin_amdgcn_readlane((el <= er) ? 1 : 0, fl) != 0;
        const uint64_t far = nearLeft ? R : L;
        pkN()[sp] = (N << 1) | (nearLeft ? 1 : 0);
        pkM()[sp] = far;
        if (sp < PK_LDS && in_mask_t<MASKOPS<F>>(far)) pkT()[sp * 64 + __lane_id()] = nearLeft ? er : el;
        sp++;
#if RT_NF_CODE
        curCode = (N << 1) | (nearLeft ? 0 : 1);
        act = nearLeft ? L : R;
        N = nearLeft ? cl.ref : cr.ref;
      } else if (L) {
        curCode = N << 1; act = L; N = cl.ref;
      } else if (R) {
        curCode = (N << 1) | 1; act = R; N = cr.ref;
      } else {
        N = INT32_MAX;
      }
      if (N != INT32_MAX) continue;
#else
        cur = nearLeft ? cl : cr;
        act = nearLeft ? L : R;
      } else if (L) {
        cur = cl; act = L;
      } else if (R) {
        cur = cr; act = R;
      } else {
        N = INT32_MAX;
      }
      if (N != INT32_MAX) { N = cur.ref; continue; }
#endif
    } else {  // a leaf: a run of triangles in leaf order
      const int32_t c = ~N;
      const int32_t st = (c >> 5) & LEAF_RUN_MAXSTART, cnt = c & 31;
      if (CNT && in_mask_t<MASKOPS<F>>(act)) { ct.c[C_LEAF]++; ct.c[C_MEMBER] += cnt; }
#if RT_F32_TRI
      const TriRayF trf = tri_ray_f32(ao, ad);
#endif
      for (int i = 0; i < cnt; ++i) {
        PKSTAT(P_CT_STEP, act);
        WCNT(C_WTRI, 1);
        bool need = in_mask_t<MASKOPS<F>>(act);
        if (CNT && need) ct.c[C_TRI]++;
#if RT_F32_TRI
        {
          const TriFR TF = sload_trif(S.triF + st + i);
          if (need) need = !tri_f32_out(TF, trf);
          if (!__ballot(need)) continue;
        }
#endif
        const TriG T = sload_tri(S.tri + st + i);
        if (need) {
          double t;
          int args;
          const bool th = tri_test(T, ao, ad, t, args, LimNF{bt, best.t});
          PKSTAT_HIT(P_CTH_STEP, th);
          if (th && (t < bt || (t == bt && st + i < bref))) {
            bt = t;
            bref = st + i;
            // the ray enters the leaf box (the reference's slab arithmetic) clearly before t
            double te;
#if RT_NF_CODE
            const ChildBox cur = sload_child(S.node + (curCode >> 1), curCode & 1);
#endif
            inside = slab_exact(cur.mn, cur.mx, ao, ad, ri, te) && te < t - t * 0x1p-40;
          }
        }
      }
    }
    // pop the nearest pending child that some lane still needs
    N = INT32_MAX;
    while (sp > 0) {
      --sp;
      const int32_t code = uni(pkN()[sp]);
      uint64_t M = uni64(pkM()[sp]);
      const NodeD* pn = S.node + (code >> 1);
      bool keep = false;
      if (in_mask_t<MASKOPS<F>>(M)) {
        const double bnd = fmin(best.t, bt), lim = fmin(bnd + bnd * 0x1p-40, 0x1p1000);  // a miss (DMAX) never passes
        double e;
        if (sp < PK_LDS) {
          e = pkT()[sp * 64 + __lane_id()];
        } else {
          const ChildBox cb = sload_child(pn, code & 1);
          e = entry_grown(cb.mn, cb.mx, sload_slack(pn, code & 1), ao, ri.y);
        }
        keep = e <= lim;
      }
      M = __ballot(keep);
#if RT_NF_CODE
      if (M) { curCode = code; act = M; N = sload_ref(pn, code & 1); break; }
#else
      if (M) { cur = sload_child(pn, code & 1); act = M; N = cur.ref; break; }
#endif
    }
    if (N == INT32_MAX) break;
  }
  const bool win = bt < best.t;
  const bool fb = win && !inside;
  if (__ballot(fb)) {  // fat-edge winners outside their leaf box: the reference traversal decides
    if (fb) accel_closest_pk<CNT, F>(S, A, ao, ad, ri, w, k, hc, best, outer, ct);
  }
  if (win && !fb) {
    best.t = bt; best.ref = bref; best.top = (int16_t)hc.top; best.inAcc = 1; best.inst = hc.inst;
    best.ver = w.ver; best.iver = 0;
    if (bt < outer) outer = bt;
  }
}

// myInstance.intersectCheck (mySceneObject.java:119-124): the named object tested with
// the instance ray (instance CTM inverse x w) as both of its rays; for a named accel
// that ray is re-normalised in place by its leaves. `local` receives the minimal t.
template <bool CNT, uint32_t F>
DEVI void inst_closest(const SceneD& S, int32_t ii, WRay& w, const Key& k, int top, Best& best, double& local,
                       Counters& ct) {
  if constexpr ((F & FT_INST) != 0) {
    const PrimD& I = S.prim[ii];
    const double* inv = S.xf[I.xf].inv;
    WRay wi;
    wi.o = xpt(inv, w.o);
    wi.d = xvec(inv, w.d);
    wi.d0 = wi.d;
    wi.ver = 0; wi.stable = false; wi.moved = false;
    const HitCtx hc{top, ii, w.ver};
    if (I.flags & PF_INST_ACCEL) {
      const AccelD& A = S.accel[I.pad[0]];
      if (CNT) { ct.c[C_ROOT]++; ct.c[C_BOX]++; }
      const RayInv ri = ray_inv(wi.o, wi.d, S.fastSlab & SCENE_FAST_SLAB);
      if (!box_hit<MASKOPS<F>>(A.bmin, A.bmax, wi.o, wi.d, ri)) return;  // myAccelStruct.intersectCheck root box
      accel_closest<CNT, F, true>(S, A, wi.o, wi.d, ri, wi, k, hc, best, local, ct);
    } else {
      double t;
      int args;
      const int32_t ref = I.pad[0];
      if (test_ref<CNT, F>(S, ref, wi.o, wi.d, k, t, args, ct, LimClosest{local, best.t})) {
        if (t < local) local = t;
        if (t < best.t) {
          best.t = t; best.ref = ref; best.top = (int16_t)top; best.inAcc = 0; best.inst = ii;
          best.ver = w.ver; best.iver = 0;
        }
      }
    }
  }
}

// Top-level culling by world bounding spheres (trace.hip top_bounds, inflated 1e-6): true
// when the world ray (w.o, w.d, |w.d| = 1 after renorm) misses the sphere or enters it
// beyond `lim` (the running best hit / the shadow distance), so the entry's own test could
// not produce a hit the reference keeps. The sphere contains every point the test can
// accept by a margin far above the test's rounding, so the outcome is the reference's; RNG
// draws are keyed, not a stream (Q23), so skipping a test shifts nothing else. A BVH / list
// entry re-normalises the ray in place in its leaves (myRay.java:93), so it is skipped only
// for a ray that re-normalisation no longer changes (WRay.stable): callers check that.
template <bool PK>
DEVI bool top_culled(const SceneD& S, int i, const WRay& w, double lim) {
  const double* b = S.topBound + 4 * i;
  const double R = PK ? sload(b + 3) : b[3];
  if (!(R > 0)) return false;
  const V c = PK ? mk(sload(b), sload(b + 1), sload(b + 2)) : mk(b[0], b[1], b[2]);
  const V oc = mk(c.x - w.o.x, c.y - w.o.y, c.z - w.o.z);
  const double tca = dot(oc, w.d), oc2 = dot(oc, oc);
  const double d2 = oc2 - tca * tca, R2 = R * R;
  if (d2 - R2 > 1e-9 * (oc2 + R2)) return true;  // misses the sphere
  // enters it beyond lim: tca - sqrt(R2 - d2) > L, L = lim + 1e-9 (|lim| + |oc| + R), with
  // |oc| <= (oc2 + 1) / 2 and the squares compared with slack (no square roots)
  const double L = lim + 1e-9 * (fabs(lim) + 0.5 * (oc2 + 1) + R), a = tca - L, h2 = fmax(R2 - d2, 0.0);
  return a > 0 && a * a > h2 * (1 + 1e-12) + 1e-12 * (oc2 + R2);
}

// ---------------------------------------------------------------------------
// Wave-level shadow candidates (SCENE_WAVE_CULL, round 3). calcShadow (myScene.java:879-885)
// tests every objList entry; the per-lane cull (top_culled) skips an entry whose bounding sphere
// the lane's ray misses, but pays that sphere test for every entry, lane and shadow ray -- C4's
// 21 entries x 6 lights made the shadow scan ~40 % of its wave time. For a point / spot light
// whose CTM is the identity (LightD.pad[0] = 1, set by the host), lane l's shadow ray runs along
// nrmz(origin - p_l) for |p_l - origin| (calcShadowColor :98-121), so a blocking hit
// (0 < t < dist - 1e-7, Q7) lies on the segment [p_l, origin]; every such segment lies within sp
// of [p_f, origin], f the wave's first shading lane and sp the spread of the hit points (max-norm
// x sqrt 3: the point at fraction s of lane l's segment is within |p_l - p_f| of the point at
// fraction s of f's). An entry whose bounding sphere (radius R, trace.hip top_bounds) stays
// farther than R + sp from [p_f, origin] therefore holds no blocker for any lane of the wave.
// Once per shading step (light_sum), the shading lanes test the (light, entry) pairs round robin
// -- one pass for C4's 6 x 21 -- and OR each light's candidate bits into LDS (the compacted-shadow
// group area, idle in this path); shadowed_ then jumps from candidate to candidate. The test is a
// superset of the capsule (line distance <= Q and projection within [-Q, |v| + Q]) with slack far
// above its rounding. Quads, planes and top-level triangles (no bounding sphere) are skipped when
// the wave's segments stay strictly on one side of their world plane(s) (trace.hip top_planes,
// after the spheres in topBound); instances, disk or transformed lights and lights past the 8th
// keep every entry. A skipped entry's in-place
// re-normalisation of the ray (myRay.java:93) is still applied, in order, before the next test,
// so every test sees the reference's direction: images are bit-identical (GPU tests), only the
// entries visited change. Measured: C4 582 -> 501 ms with the spheres, 472 ms with the plane
// sides (the per-light form 561 ms; as a real call 711-792 ms: it is inlined; the same test for
// the closest-hit scan of a step's rays, 521 ms: dropped; profiles/r03n_*, r03o_*, r03r_*).
#ifndef RT_WAVE_CULL
#define RT_WAVE_CULL 1
#endif
// variants with the wave-level shadow cull: non-triangle primitives, no photon map (C4's); the
// host enables it per launch (SCENE_WAVE_CULL: ntop <= 64, culling on)
#ifndef RT_WC_TRI  // also in the triangles-only variants (C3's: two ground triangles and a BVH)
#define RT_WC_TRI 0
#endif
template <uint32_t F>
static constexpr bool WAVE_CULL = RT_WAVE_CULL && ((F & FT_PRIM) != 0 || RT_WC_TRI) && (F & FT_PHOTON) == 0;
DEVI double rdl(double v, int L) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, L), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), L);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
DEVI lds_u64* wcM() { return (lds_u64*)(pkB() + LDS_BYTES + SUM_BYTES); }
// the candidate bits of lights 0..7 for the hit points p of the active lanes (wave-scope LDS
// atomics of the active lanes only: the ockl wave reductions assume no holes in the exec mask)
DEVI void step_cands(const SceneD& S, V p) {
  lds_u64* M = wcM();
  const uint64_t act = __ballot(1);
  const int f = (int)__builtin_ctzll(act);
  const V pf = mk(rdl(p.x, f), rdl(p.y, f), rdl(p.z, f));
  // the spread: sp >= 0 (or NaN), so its bits order as its value; a NaN makes every entry a candidate
  double sp = fmax(fmax(fabs(p.x - pf.x), fabs(p.y - pf.y)), fabs(p.z - pf.z));
  M[0] = 0;
  __hip_atomic_fetch_max(M, __builtin_bit_cast(uint64_t, sp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  sp = __builtin_bit_cast(double, __hip_atomic_load(M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT)) * 1.7320508075688776;
  const int nl = S.nlight < GRP_MAX ? S.nlight : GRP_MAX, nt = S.ntop, np = nl * nt;
  for (int q = 0; q < nl; ++q) M[q] = 0;
  const int nact = __popcll(act);
  const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  const uint32_t rcp = (1u << 20) / (uint32_t)nt + 1;  // q / nt exactly for q < 512, nt <= 64
  const double pn = fmax(fmax(fabs(pf.x), fabs(pf.y)), fabs(pf.z));
  for (int q0 = 0; q0 < np; q0 += nact) {
    const int q = q0 + rank;
    if (q < np) {
      const int li = (int)(((uint32_t)q * rcp) >> 20), i = q - li * nt;
      const LightD& L = S.light[li];
      const double* b = S.topBound + 4 * i;
      const double R = b[3];
      bool cand = true;
      if (L.pad[0] == 1 && !(R > 0)) {  // a quad / plane: the segments strictly on one side of its plane(s)
        const double* pl = S.topBound + 4 * nt + 8 * i;
        const double m = 1e-6 * (1 + pn + fmax(fmax(fabs(L.origin[0]), fabs(L.origin[1])), fabs(L.origin[2])));
        bool off = pl[0] != 0 || pl[1] != 0 || pl[2] != 0;
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const double* q = pl + 4 * o;
          const double sP = q[0] * pf.x + q[1] * pf.y + q[2] * pf.z + q[3];
          const double sL = q[0] * L.origin[0] + q[1] * L.origin[1] + q[2] * L.origin[2] + q[3];
          const double mm = m * (1 + fabs(q[3]));
          off = off && ((sP - sp > mm && sL > mm) || (sP + sp < -mm && sL < -mm));
        }
        cand = !off;
      } else if (L.pad[0] == 1) {
        const V v = mk(L.origin[0] - pf.x, L.origin[1] - pf.y, L.origin[2] - pf.z);
        const double vv = v.x * v.x + v.y * v.y + v.z * v.z, vl = sqrt(vv);
        const V w = mk(b[0] - pf.x, b[1] - pf.y, b[2] - pf.z);
        const double wv = w.x * v.x + w.y * v.y + w.z * v.z, ww = w.x * w.x + w.y * w.y + w.z * w.z;
        const double Q = (R + sp + 1e-9 * (1 + vl + sp + pn + R)) * (1 + 1e-9), Q2 = Q * Q;
        const double perp = ww * vv - wv * wv, slackP = 1e-9 * (ww * vv + Q2 * vv);
        const double slackT = 1e-9 * (sqrt(ww) * vl + vv), qv = Q * vl;
        // "far" from comparisons that are false on NaN: a NaN / Inf segment stays a candidate
        cand = !(perp > Q2 * vv + slackP || wv < -qv - slackT || wv > vv + qv + slackT);
      }
      if (cand) __hip_atomic_fetch_or(M + li, 1ull << i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
}
DEVI void step_cands_all() {
  for (int q = 0; q < GRP_MAX; ++q) wcM()[q] = ~0ull;
}
// light li's candidate bits, read where the scan starts (no register holds them before it)
DEVI uint64_t step_cand(int li) { return li < GRP_MAX ? uni64(*(volatile lds_u64*)(wcM() + li)) : ~0ull; }

// findClosestRayHit (myScene.java:888-903): objList scan, TreeMap keeps the first of equal t
#ifndef RT_PACKET
#define RT_PACKET 1
#endif
static constexpr bool PACKET = RT_PACKET != 0;  // render kernel: packet traversal
// shade_node keeps the hit's normal / view direction / texture colour in the LDS slots while
// its shadow rays are traced (stash() above); RT_STASH_SHADE=0 keeps them in registers
#ifndef RT_STASH_SHADE
#define RT_STASH_SHADE 1
#endif
static constexpr bool STASH_SHADE = PACKET && RT_STASH_SHADE != 0 && PK_LDS >= SL_N;
// PK: packet traversal of the BVHs (render kernel; the lanes of a wave are coherent)
// experiment (default off): when at least RT_LANE_DIV lanes' rays point away from the wave's first
// ray (cosine below RT_LANE_DIV_COS), the BVHs are traversed lane by lane (accel_closest: the
// reference order, per-lane stacks) instead of as one packet walking the union of the lanes' paths
#ifndef RT_LANE_DIV
#define RT_LANE_DIV 0
#endif
#ifndef RT_LANE_DIV_COS
#define RT_LANE_DIV_COS 0.9
#endif
template <bool CNT, uint32_t F, bool PK = false>
DEVI Best closest(const SceneD& S, WRay& w, const Key& k, Counters& ct) {
  PROF_T0(t_all);
  Best best = miss();
  bool lanes = false;
  if constexpr (PK && RT_LANE_DIV > 0) {
    const int f = (int)__builtin_ctzll(__ballot(1));
    const double c = w.d.x * rdl(w.d.x, f) + w.d.y * rdl(w.d.y, f) + w.d.z * rdl(w.d.z, f);
    const int nfar = __popcll(__ballot(!(c >= RT_LANE_DIV_COS))), nact = __popcll(__ballot(1));
    lanes = RT_LANE_DIV == 1 ? (nfar >= 2 && 2 * nfar >= nact) : nfar >= RT_LANE_DIV;
  }
  for (int i = 0; i < S.ntop; ++i) {
    TopD tp = PK ? sload_top(S.top + i) : S.top[i];
    if (CNT) ct.c[C_TOP]++;
    renorm(w);
    if ((F & FT_INST) && tp.kind == TOP_INST) {
      double local = best.t;
      inst_closest<CNT, F>(S, tp.idx, w, k, i, best, local, ct);
      continue;
    }
    if ((((F & FT_PRIM) && tp.kind == TOP_PRIM) || (tp.kind == TOP_ACCEL && w.stable)) && top_culled<PK>(S, i, w, best.t))
      continue;
    V o, d;
    if (PK) {  // wave-uniform records: scalar loads
      double inv[12];
      sload_inv(S.xf + tp.xf, inv);
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    } else {
      const double* inv = S.xf[tp.xf].inv;
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    }
    if (tp.kind == TOP_ACCEL) {
      const AccelD A = PK ? sload_accel(S.accel + tp.idx) : S.accel[tp.idx];
      if (CNT) { ct.c[C_ROOT]++; ct.c[C_BOX]++; }
      RayInv ri = ray_inv(o, d, S.fastSlab & SCENE_FAST_SLAB);
      if (!box_hit<MASKOPS<F>>(A.bmin, A.bmax, o, d, ri)) continue;
      w.moved = false;
      double local = DMAX;
      PROF_T0(t_acc);
      if (RT_LANE_DIV > 0 && lanes)
        accel_closest<CNT, F, false>(S, A, o, d, ri, w, k, HitCtx{i, -1, 0}, best, local, ct);
      else if (PK && NEAREST_FIRST && (F & (FT_PHOTON | (RT_NF_TRANS ? 0 : FT_TRANS))) == 0 && (S.fastSlab & SCENE_NEAREST_FIRST) &&
          (A.flags & ACCEL_NEAREST) &&
          !__ballot(!(w.stable && ri.fast)))
        accel_closest_nf<CNT, F>(S, A, o, d, ri, w, k, HitCtx{i, -1, 0}, best, local, ct);
      else if (PK) accel_closest_pk<CNT, F>(S, A, o, d, ri, w, k, HitCtx{i, -1, 0}, best, local, ct);
      else accel_closest<CNT, F, false>(S, A, o, d, ri, w, k, HitCtx{i, -1, 0}, best, local, ct);
      PROF_ADD(t_acc, R_CLOSEST_ACCEL);
    } else {
      int32_t ref = tp.kind == TOP_TRI ? tp.idx : ~tp.idx;
      double t;
      int args;
      if (test_ref_u<CNT, F, PK>(S, ref, o, d, k, t, args, ct, LimClosest{best.t, best.t}) && t < best.t) {
        best.t = t; best.ref = ref; best.top = (int16_t)i; best.inAcc = 0; best.ver = w.ver; best.inst = -1; best.iver = 0;
      }
    }
  }
  PROF_ADD(t_all, R_CLOSEST);
  return best;
}

// any-hit: mySceneObject/myBBox/myGeomList/myBVH.calcShadowHit (mySceneObject.java:33-38,
// myGeomBase.java:166-170, 268-277, 397-404): blocked iff hit && dist - t > 1e-7
template <bool CNT, bool A2 = (RT_APX2 != 0)>
DEVI bool shadow_box(const double* mn, const double* mx, V o, V d, const RayInv& ri, double dist, Counters& ct) {
  if (CNT) ct.c[C_BOX]++;
  return box_shadow<A2>(mn, mx, o, d, ri, dist);
}
template <bool CNT, uint32_t F>
DEVI bool inst_any(const SceneD& S, int32_t ii, const WRay& w, const Key& k, double dist, Counters& ct);

template <bool CNT, uint32_t F, bool INST, bool PK = false>
DEVI bool leaf_any(const SceneD& S, int32_t leaf, int accXf, V ao, V ad, WRay& w, const Key& k, double dist, Counters& ct) {
  const LeafR lf = leaf_of<PK>(S, leaf);
  if (CNT) { ct.c[C_LEAF]++; ct.c[C_MEMBER] += lf.count; }
  // the fp32 triangle pre-test (members in the accel's CTM)
  constexpr bool TF32 = PK && RT_F32_TRI != 0 && ((F & FT_PHOTON) == 0 || RT_F32_TRI_PH_ANY != 0);
  TriRayF trf;
  if constexpr (TF32) trf = tri_ray_f32(ao, ad);
  for (int i = 0; i < lf.count; ++i) {
    if (PK) PKSTAT(P_AT_STEP, __ballot(1));
    int32_t ref = leaf_member<PK>(S, lf, i);
    renorm(w);
    if constexpr (!INST && (F & FT_INST) != 0) {
      if (is_inst<F>(S, ref)) {  // myInstance.calcShadowHit
        if (inst_any<CNT, F>(S, ~ref, w, k, dist, ct)) return true;
        continue;
      }
    }
    int xf = ref_xf_u<F, PK>(S, ref);
    V o, d;
    if (xf == accXf && !w.moved) { o = ao; d = ad; }
    else if (PK && (RT_ULOAD & 1)) {  // xf is wave-uniform here (ref_xf_u): the inverse as scalar loads
      double inv[12];
      sload_inv(S.xf + xf, inv);
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    } else { const double* inv = S.xf[xf].inv; o = xpt(inv, w.o); d = xvec(inv, w.d); }
    double t;
    int args;
    bool th;
    if (TF32 && (!(F & FT_PRIM) || ref >= 0) && xf == accXf && !w.moved) {  // test_ref_u's triangle case
      if (CNT) ct.c[C_TRI]++;
      WCNT(C_WTRI, 1);
      const TriFR TF = sload_trif(S.triF + ref);
      th = false;
      if (!tri_f32_out(TF, trf)) {
        const TriG T = sload_tri(S.tri + ref);
        th = tri_test(T, o, d, t, args, LimShadow{dist}) && (dist - t) > EPS;
      }
    } else {
      th = test_ref_u<CNT, F, PK>(S, ref, o, d, k, t, args, ct, LimShadow{dist}) && (dist - t) > EPS;
    }
    if (PK) PKSTAT_HIT(P_ATH_STEP, th);
    if (th) return true;
  }
  return false;
}
template <bool CNT, uint32_t F, bool INST>
DEVI bool accel_any(const SceneD& S, const AccelD& A, V ao, V ad, WRay& w, const Key& k, double dist, Counters& ct) {
  RayInv ri = ray_inv(ao, ad, S.fastSlab & SCENE_FAST_SLAB);
  NStackT<INST ? 0 : STK_LDS> st;
  int sp = 0;
  int32_t N = A.root;
  // leafVals.calcShadowHit tests its own box first; myBVH.calcShadowHit (internal) does not
  if (N < 0 && !shadow_box<CNT>(A.bmin, A.bmax, ao, ad, ri, dist, ct)) return false;
  while (true) {
    if (N >= 0) {  // internal: push (right child pending), go left if its box is hit
      const NodeD& nd = S.node[N];
      if (CNT) { ct.c[C_NODE]++; ct.c[C_WNODE]++; }
      st.setN(sp++, N);
      if (shadow_box<CNT>(nd.lmin, nd.lmax, ao, ad, ri, dist, ct)) { N = nd.left; continue; }
    } else if (N != INT32_MAX) {
      if (leaf_any<CNT, F, INST>(S, ~N, INST ? -1 : A.xf, ao, ad, w, k, dist, ct)) return true;
      if (INST && w.moved) { ad = w.d; ri = ray_inv(ao, ad, S.fastSlab & SCENE_FAST_SLAB); w.moved = false; }
    }
    N = INT32_MAX;
    while (sp > 0) {
      const NodeD& pn = S.node[st.getN(--sp)];
      if (shadow_box<CNT>(pn.rmin, pn.rmax, ao, ad, ri, dist, ct)) { N = pn.right; break; }
    }
    if (N == INT32_MAX) return false;
  }
}
// accel_any<INST = false> as a packet traversal; a lane leaves the packet when blocked.
// Both child boxes of a node are loaded (one scalar batch) and tested when it is pushed:
// a box test is a pure function of (ray, box, dist), so testing the right box early
// changes nothing but removes the unwind step's dependent scalar load. The frame keeps
// the right child, the lanes in the node's subtree (M) and those whose right box is hit
// (R); at the unwind the lanes still unblocked in R descend. The counting kernel counts
// the right-box test at the unwind, for the lanes in M still unblocked, as accel_any does.
// Nearest-first (RT_ANY_NEAR, rays the re-normalisation no longer changes): when both child
// boxes are hit, the child the ray enters first is visited first. Whether a shadow ray is blocked
// does not depend on the order the reachable leaves are tested in (a stable ray's direction no
// longer changes), so only the work to the first blocker changes.
#ifndef RT_ANY_NEAR
#define RT_ANY_NEAR 1
#endif
template <bool CNT, uint32_t F>
DEVI bool accel_any_pk(const SceneD& S, const AccelD& A, V ao, V ad, WRay& w, const Key& k, double dist, Counters& ct) {
  const RayInv ri = ray_inv(ao, ad, S.fastSlab & SCENE_FAST_SLAB);
  // (C3's triangles-only variant gains 2 %; the transparent variants lose as much: not there)
  const bool nearf = RT_ANY_NEAR && (RT_AN_TRANS || (F & FT_TRANS) == 0) && (S.fastSlab & SCENE_NEAREST_FIRST) && !__ballot(!w.stable);
  // the fp32 box pre-test (box32): a shadow box decision -- hit and (dist - entry) - EPS > 0 -- is
  // settled when the entry is certain to lie clear of dist - EPS (bracketed here by 2^-20 of it)
  constexpr bool F32 = RT_F32_BOX && RT_F32_SHADOW && ((F & FT_TRANS) != 0 ? RT_F32_SHADOW_TRANS : RT_F32_SHADOW_OPAQUE);
  const bool f32 = F32 && ri.fast;
  // RT_F32_SH_LAZY: only the margin's two ray terms and the distance bracket live across the
  // traversal; the fp32 ray itself is rebuilt from the fp64 one (live anyway) at each node -- fewer
  // registers held through the shading code the traversal is inlined into
  RayF rf;
  float dLo = 0, dHi = 0;
  if constexpr (F32) {
    rf = ray_f32(ao, ri, fmax(fmax(fabs(ri.y[0]), fabs(ri.y[1])), fabs(ri.y[2])));
    const double dm = dist - EPS;
    dLo = (float)(dm - fabs(dm) * 0x1p-20);
    dHi = (float)(dm + fabs(dm) * 0x1p-20);
  }
  PkStack st;
  int sp = 0;
  uint64_t act = __ballot(1);
  uint64_t alive = act;
  bool blocked = false;
  int32_t N = uni(A.root);
  const int32_t axf = A.xf;
  // leafVals.calcShadowHit tests its own box first; myBVH.calcShadowHit (internal) does not
  if (N < 0) {
    bool hb = false;
    if (in_mask_t<MASKOPS<F>>(act)) hb = shadow_box<CNT, MASKOPS<F>>(A.bmin, A.bmax, ao, ad, ri, dist, ct);
    act = __ballot(hb);
    if (!act) return false;
  }
  while (true) {
    if (N >= 0) {  // internal: push (right child pending), go left with the lanes whose left box is hit
      PKSTAT(P_AB_STEP, act);
      WCNT(C_WNODE, 1);
      bool hl = false, hr = false;
      double el = DMAX, er = DMAX;
      struct { int32_t ref; } cl{0}, cr{0};
      if constexpr (F32) {
        const NodeD* nd = S.node + N;
        const NodeBoxF nb = sload_nodef(S.nodeF + N);
        cl.ref = sload_ref(nd, 0);
        cr.ref = sload_ref(nd, 1);
        bool ol = false, orr = false;
        if (in_mask_t<MASKOPS<F>>(act)) {
          if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX]++; }
          if (f32) {
            if constexpr (RT_F32_SH_LAZY != 0 && (F & FT_PHOTON) == 0) {
              const RayF r2 = ray_f32_dirs(ao, ri);
              rf.y[0] = r2.y[0]; rf.y[1] = r2.y[1]; rf.y[2] = r2.y[2];
              rf.noy[0] = r2.noy[0]; rf.noy[1] = r2.noy[1]; rf.noy[2] = r2.noy[2];
            }
            const float E = f32_margin(rf, nb.mag);
            float lo;
            const int c0 = box32(nb.b, rf, E, lo);
            if (c0 == B32_HIT && dLo > lo + 2 * E) { hl = true; el = lo; }
            else ol = !(c0 == B32_MISS || dHi < lo - 2 * E);
            const int c1 = box32(nb.b + 6, rf, E, lo);
            if (c1 == B32_HIT && dLo > lo + 2 * E) { hr = true; er = lo; }
            else orr = !(c1 == B32_MISS || dHi < lo - 2 * E);
          } else {
            ol = orr = true;
          }
        }
        if (__ballot(ol)) {  // unsettled lanes: the fp64 test
          const ChildBox c = sload_child(nd, 0);
          if (ol) hl = box_shadow_e<MASKOPS<F>>(c.mn, c.mx, ao, ad, ri, dist, el);
        }
        if (__ballot(orr)) {
          const ChildBox c = sload_child(nd, 1);
          if (orr) hr = box_shadow_e<MASKOPS<F>>(c.mn, c.mx, ao, ad, ri, dist, er);
        }
      } else {
        const ChildBox c0 = sload_child(S.node + N, 0);
        const ChildBox c1 = sload_child(S.node + N, 1);
        cl.ref = c0.ref;
        cr.ref = c1.ref;
        if (in_mask_t<MASKOPS<F>>(act)) {
          if (CNT) { ct.c[C_NODE]++; ct.c[C_BOX]++; }
          hl = box_shadow_e<MASKOPS<F>>(c0.mn, c0.mx, ao, ad, ri, dist, el);
          hr = box_shadow_e<MASKOPS<F>>(c1.mn, c1.mx, ao, ad, ri, dist, er);
        }
      }
      const uint64_t R = __ballot(hr);
      const uint64_t H = __ballot(hl);
      if (nearf && H && R) {
        const int fl = (int)__builtin_ctzll(H & R);
        if (__builtin_amdgcn_readlane((er < el) ? 1 : 0, fl)) {  // the right child first, the left pending
          st.setFrameR(sp++, 0, act, H, cl.ref);
          act = R; N = cr.ref;
          continue;
        }
      }
      if (CNT || R) st.setFrameR(sp++, 0, act, R, cr.ref);
      if (H) { act = H; N = cl.ref; continue; }
    } else if (N != INT32_MAX) {
      bool b = false;
      if (in_mask_t<MASKOPS<F>>(act)) b = leaf_any<CNT, F, false, true>(S, ~N, axf, ao, ad, w, k, dist, ct);
      if (b) blocked = true;
      alive &= ~__ballot(b);
      if (!alive) return blocked;
    }
    N = INT32_MAX;
    while (sp > 0) {
      --sp;
      if (CNT && in_mask_t<MASKOPS<F>>(st.getM(sp) & alive)) ct.c[C_BOX]++;
      const uint64_t R = st.getR(sp) & alive;
      if (R) { act = R; N = st.getC(sp); break; }
    }
    if (N == INT32_MAX) return blocked;
  }
}

// myInstance.calcShadowHit (mySceneObject.java:115-118): obj.calcShadowHit(_trans, _trans, ...)
template <bool CNT, uint32_t F>
DEVI bool inst_any(const SceneD& S, int32_t ii, const WRay& w, const Key& k, double dist, Counters& ct) {
  if constexpr ((F & FT_INST) != 0) {
    const PrimD& I = S.prim[ii];
    const double* inv = S.xf[I.xf].inv;
    WRay wi;
    wi.o = xpt(inv, w.o);
    wi.d = xvec(inv, w.d);
    wi.d0 = wi.d;
    wi.ver = 0; wi.stable = false; wi.moved = false;
    if (I.flags & PF_INST_ACCEL) return accel_any<CNT, F, true>(S, S.accel[I.pad[0]], wi.o, wi.d, wi, k, dist, ct);
    double t;
    int args;
    return test_ref<CNT, F>(S, I.pad[0], wi.o, wi.d, k, t, args, ct, LimShadow{dist}) && (dist - t) > EPS;
  }
  return false;
}
// myScene.calcShadow (myScene.java:879-885). WC: light li's wave-level candidates only
// (step_cands / step_cands_all have written them)
template <bool CNT, uint32_t F, bool PK = false, bool WC = false>
DEVI bool shadowed_(const SceneD& S, WRay& w, const Key& k, double dist, Counters& ct, int li) {
  const uint64_t cand = WC ? step_cand(li) : ~0ull;
  for (int i = 0; i < S.ntop; ++i) {
    // on to the next candidate; the skipped entries' in-place re-normalisations still apply. The
    // candidate word covers entries 0..63 (SCENE_WAVE_CULL needs ntop <= 64; otherwise it is ~0):
    // past it every entry is tested (a shift by >= 64 would wrap on the device and loop forever)
    if (WC && i < 64) {
      const uint64_t rest = cand & (~0ull << i);
      const int nx = rest ? (int)__builtin_ctzll(rest) : S.ntop;
      for (int j = i; j < nx && !w.stable; ++j) renorm(w);
      if (nx >= S.ntop) break;
      i = nx;
    }
    TopD tp = PK ? sload_top(S.top + i) : S.top[i];
    if (CNT) ct.c[C_TOP]++;
#if defined(RT_PROF_SH_NOQUAD) || defined(RT_PROF_SH_NOIMPL)  // profiling builds only: results differ
    if (tp.kind == TOP_PRIM) {
      const bool bounded = sload(S.topBound + 4 * i + 3) > 0;
#ifdef RT_PROF_SH_NOQUAD
      if (!bounded) continue;
#else
      if (bounded) continue;
#endif
    }
#endif
#ifdef RT_PROF_SH_NOACCEL
    if (tp.kind == TOP_ACCEL) continue;
#endif
    renorm(w);
    if ((F & FT_INST) && tp.kind == TOP_INST) {
      if (inst_any<CNT, F>(S, tp.idx, w, k, dist, ct)) return true;
      continue;
    }
    if ((((F & FT_PRIM) && tp.kind == TOP_PRIM) || (tp.kind == TOP_ACCEL && w.stable)) && top_culled<PK>(S, i, w, dist))
      continue;
#ifdef RT_PROF_SH_SCANONLY  // profiling builds only: the scan (re-normalisation, culling) without the tests
    continue;
#endif
    V o, d;
    if (PK) {  // wave-uniform records: scalar loads
      double inv[12];
      sload_inv(S.xf + tp.xf, inv);
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    } else {
      const double* inv = S.xf[tp.xf].inv;
      o = xpt(inv, w.o); d = xvec(inv, w.d);
    }
    if (tp.kind == TOP_ACCEL) {
      if (CNT) ct.c[C_ROOT]++;
      w.moved = false;
      PROF_T0(t_acc);
      const bool blk = PK ? accel_any_pk<CNT, F>(S, sload_accel(S.accel + tp.idx), o, d, w, k, dist, ct)
                          : accel_any<CNT, F, false>(S, S.accel[tp.idx], o, d, w, k, dist, ct);
      PROF_ADD(t_acc, R_SHADOW_ACCEL);
      if (blk) return true;
    } else {
      int32_t ref = tp.kind == TOP_TRI ? tp.idx : ~tp.idx;
      double t;
      int args;
      if (test_ref_u<CNT, F, PK>(S, ref, o, d, k, t, args, ct, LimShadow{dist}) && (dist - t) > EPS) return true;
    }
  }
  return false;
}
#ifdef RT_SHADOW_NOINLINE  // experiment: the shadow scan as a real call
#define SHADOW_FN __device__ __attribute__((noinline))
#else
#define SHADOW_FN DEVI
#endif
template <bool CNT, uint32_t F, bool PK = false, bool WC = false>
SHADOW_FN bool shadowed(const SceneD& S, WRay& w, const Key& k, double dist, Counters& ct, int li = 0) {
  PROF_T0(t_all);
  const bool r = shadowed_<CNT, F, PK, WC>(S, w, k, dist, ct, li);
  PROF_ADD(t_all, R_SHADOW);
  return r;
}

// ---------------------------------------------------------------------------
// hit record (myRay.objHit :119-125, rayHit ctor :147-161, reCalcCTMHitNorm :168-175)
struct HitRec {
  V hitLoc, fwd, nrm, dw;
  int32_t mat, args, type, ref;
  uint32_t key;
};
template <uint32_t F>
DEVI HitRec make_hit(const SceneD& S, const Best& b, const WRay& w, const Key& k) {
  HitRec h;
  int32_t ref = b.ref;
  V dw = w.d0;  // direction at the winning test: d0 re-normalised `ver` times
  for (uint32_t i = 0; i < b.ver; ++i) dw = nrmz(dw);
  int xf, xfc;
  if (!(F & FT_PRIM) || ref >= 0) { const TriD& T = S.tri[ref]; xf = T.xf; xfc = T.xfc; h.mat = T.mat; h.key = T.key; h.type = PT_TRI; }
  else { const PrimD& P = S.prim[~ref]; xf = P.xf; xfc = P.xfc; h.mat = P.mat; h.key = P.key; h.type = P.type; }
  h.ref = ref;
  V ro = w.o;  // the ray the primitive's caller passed as `_ray` (its direction is rawRayDir)
  int hitXf = -1;  // CTM of the hit record when it is not the primitive's own / accel one
  bool direct = false;  // the primitive was tested with `ro, dw` itself (instanced primitive)
  if ((F & FT_INST) && b.inst >= 0) {  // myInstance: the instance ray, re-normalised `iver` times
    const PrimD& I = S.prim[b.inst];
    const XformD& XI = S.xf[I.xf];
    ro = xpt(XI.inv, w.o);
    dw = xvec(XI.inv, dw);
    for (uint32_t i = 0; i < b.iver; ++i) dw = nrmz(dw);
    if (I.mat >= 0) h.mat = I.mat;  // useInstShader
    direct = !(I.flags & PF_INST_ACCEL);
    // reCalcCTMHitNorm by the list holding the instance (sierpinski), else the instance CTM
    // (instanced primitive) or the named accel's leaf CTM (xfc, as for any accel hit)
    hitXf = (I.xfc >= 0) ? I.xfc : (direct ? I.xf : -1);
  }
  const XformD& X = S.xf[xf];
  V tro = direct ? ro : xpt(X.inv, ro), trd = direct ? dw : xvec(X.inv, dw);
  double t = b.t, tt;
  int args = 0;
  if (!(F & FT_PRIM) || ref >= 0) {
    // a triangle's only hit argument is its orientation: planar_test's st = (nA . d > 0), the
    // same product of the same operands as in the winning test
    const V nA = ld3(S.tri[ref].n);
    args = dot(nA, trd) > 0 ? 1 : 0;
  } else {
    Counters dummy;
    test_ref<false, F>(S, ref, tro, trd, k, tt, args, dummy);  // recompute args (deterministic)
  }
  h.args = args;
  V p = mk(trd.x * t + tro.x, trd.y * t + tro.y, trd.z * t + tro.z);
  h.hitLoc = p;
  V n;
  if (!(F & FT_PRIM) || ref >= 0) {  // planar getNormalAtPoint: the stored N, normalised again
    V nA = ld3(S.tri[ref].n);
    n = args ? mk(-nA.x, -nA.y, -nA.z) : nA;
    n = nrmz(n);
  } else {
    const PrimD& P = S.prim[~ref];
    switch (P.type) {
      case PT_QUAD:
      case PT_PLANE: n = nrmz(args ? ld3(P.a + 15) : ld3(P.a + 12)); break;
      case PT_SPHERE:
      case PT_MSPHERE: {  // getNormalAtPoint uses the static origin (myImpObject.java:68-74)
        n = nrmz(mk(p.x - P.a[0], p.y - P.a[1], p.z - P.a[2]));
        if (P.flags & 1) n = mk(n.x * -1.0, n.y * -1.0, n.z * -1.0);
        break;
      }
      case PT_HCYL: {
        n = (args == 1) ? mk(P.a[0] - p.x, 0, P.a[2] - p.z) : mk(p.x - P.a[0], 0, p.z - P.a[2]);
        n = nrmz(n);
        if (P.flags & 1) n = mk(n.x * -1, n.y * -1, n.z * -1);
        break;
      }
      case PT_CYL: {
        n = (args >= 2) ? mk(p.x - P.a[0], 0, p.z - P.a[2]) : ld3(P.a + 8 + 4 * args);
        n = nrmz(n);
        if (P.flags & 1) n = mk(n.x * -1, n.y * -1, n.z * -1);
        break;
      }
      default: {  // box plane normals (myGeomBase.java:175-186)
        const double tab[7][3] = {{-1, 0, 0}, {0, -1, 0}, {0, 0, -1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, -1}};
        int a = (args >= 0 && args < 6) ? args : 6;
        n = mk(tab[a][0], tab[a][1], tab[a][2]);
      }
    }
  }
  const XformD& M = (hitXf >= 0) ? S.xf[hitXf] : (b.inAcc && xfc >= 0) ? S.xf[xfc] : X;  // Q4: accel CTM x object CTM
  h.fwd = xpt(M.g, p);
  h.nrm = nrmz(xvec(M.adj, n));
  h.dw = ((F & FT_PRIM) && h.type == PT_BOX) ? xvec(X.g, trd) : dw;
  return h;
}

// ---------------------------------------------------------------------------
// Perlin noise (float), DistRayTracer.java:234-310
DEVI int pm(int i) { return c_perm[i & 255]; }
DEVI int ffl(float x) { return x > 0 ? (int)x : (int)x - 1; }
DEVI float gd(int g, float x, float y, float z) { return c_grad3[g][0] * x + c_grad3[g][1] * y + c_grad3[g][2] * z; }
DEVI float fmx(float a, float b, float t) { return (1 - t) * a + t * b; }
DEVI float fade(float t) { return t * t * t * (t * (t * 6 - 15) + 10); }
DEVI float noise3(float x, float y, float z) {
  int X = ffl(x), Y = ffl(y), Z = ffl(z);
  x = x - X; y = y - Y; z = z - Z;
  X = X & 255; Y = Y & 255; Z = Z & 255;
  int g000 = pm(X + pm(Y + pm(Z))) % 12, g001 = pm(X + pm(Y + pm(Z + 1))) % 12;
  int g010 = pm(X + pm(Y + 1 + pm(Z))) % 12, g011 = pm(X + pm(Y + 1 + pm(Z + 1))) % 12;
  int g100 = pm(X + 1 + pm(Y + pm(Z))) % 12, g101 = pm(X + 1 + pm(Y + pm(Z + 1))) % 12;
  int g110 = pm(X + 1 + pm(Y + 1 + pm(Z))) % 12, g111 = pm(X + 1 + pm(Y + 1 + pm(Z + 1))) % 12;
  float n000 = gd(g000, x, y, z), n100 = gd(g100, x - 1, y, z), n010 = gd(g010, x, y - 1, z), n110 = gd(g110, x - 1, y - 1, z);
  float n001 = gd(g001, x, y, z - 1), n101 = gd(g101, x - 1, y, z - 1), n011 = gd(g011, x, y - 1, z - 1), n111 = gd(g111, x - 1, y - 1, z - 1);
  float u = fade(x), v = fade(y), w = fade(z);
  return fmx(fmx(fmx(n000, n100, u), fmx(n010, n110, u), v), fmx(fmx(n001, n101, u), fmx(n011, n111, u), v), w);
}

DEVI V texel(const SceneD& S, const TexD& T, long i) {  // myColor(int)
  long n = (long)T.w * T.h;
  if (i < 0) i = 0;
  if (i >= n) i = n - 1;
  uint32_t c = S.texel[T.off + i];
  return mk(((c >> 16) & 0xFF) / 255.0, ((c >> 8) & 0xFF) / 255.0, (c & 0xFF) / 255.0);
}
DEVI V lerpc(V a, double t, V b) {  // myColor.interpColor (clamped <= 1)
  return mk(jmin(1, a.x + t * (b.x - a.x)), jmin(1, a.y + t * (b.y - a.y)), jmin(1, a.z + t * (b.z - a.z)));
}

// myImageTexture.getTextureColor (myTextureHandler.java:84-103) + findTxtrCoords
template <bool CNT>
DEVI V image_color(const SceneD& S, const HitRec& h, const Key& k, const TexD& T, Counters& ct) {
  double u = 0, v = 0;
  V p = h.hitLoc;
  if (h.type == PT_SPHERE || h.type == PT_MSPHERE) {  // mySphere.findTextureU/V (myImpObject.java:97-122)
    const PrimD& P = S.prim[~h.ref];
    V to = sphere_center(P, k);
    double a0 = p.y - to.y, a1 = a0 / P.a[4];
    a1 = (a1 > 1) ? 1 : (a1 < -1) ? -1 : a1;
    v = (T.h - 1) * jf::acos(a1) / PI_D;
    double shWm1 = T.w - 1, z1 = p.z - to.z, q = v / (T.h - 1);
    double b0 = (p.x - to.x) / P.a[3];
    b0 = (b0 > 1) ? 1 : (b0 < -1) ? -1 : b0;
    double b1 = jf::sin(q * PI_D);
    double a2 = (fabs(b1) < EPS) ? 1 : b0 / b1;
    u = (z1 <= EPS) ? ((shWm1 * jf::acos(a2)) / TWO_PI_F + shWm1 / 2.0) : shWm1 - ((shWm1 * jf::acos(a2)) / TWO_PI_F + shWm1 / 2.0);
    u = (u < 0) ? 0 : (u > shWm1) ? shWm1 : u;
  } else if (h.type == PT_TRI || h.type == PT_QUAD || h.type == PT_PLANE) {  // barycentric (myPlanarObject.java:178-186)
    double vx[4][3], uvv[4][2];
    int nv = 3;
    if (h.type == PT_TRI) {
      const TriD& T3 = S.tri[h.ref];
      const double* tuv = S.triUV ? S.triUV + 6 * (size_t)h.ref : nullptr;
      for (int i = 0; i < 3; ++i) {
        for (int c = 0; c < 3; ++c) vx[i][c] = T3.v[i][c];
        uvv[i][0] = tuv ? tuv[2 * i] : 0;
        uvv[i][1] = tuv ? tuv[2 * i + 1] : 0;
      }
    } else {
      const PrimD& P = S.prim[~h.ref];
      nv = 4;
      for (int i = 0; i < 4; ++i) { for (int c = 0; c < 3; ++c) vx[i][c] = P.a[3 * i + c]; uvv[i][0] = P.a[20 + 2 * i]; uvv[i][1] = P.a[21 + 2 * i]; }
    }
    double w[4][3], wu[4][2];
    for (int i = 0; i < nv; ++i) {
      int s = h.args ? nv - 1 - i : i;
      for (int c = 0; c < 3; ++c) w[i][c] = vx[s][c];
      wu[i][0] = uvv[s][0]; wu[i][1] = uvv[s][1];
    }
    V P2P0 = mk(w[1][0] - w[0][0], w[1][1] - w[0][1], w[1][2] - w[0][2]);
    V P2P2 = (nv == 3) ? mk(w[0][0] - w[2][0], w[0][1] - w[2][1], w[0][2] - w[2][2])
                       : mk(w[3][0] - w[2][0], w[3][1] - w[2][1], w[3][2] - w[2][2]);
    double d0 = dot(P2P0, P2P0), d2 = dot(P2P2, P2P2), dn = -dot(P2P0, P2P2);
    double bary = 1.0 / ((d0 * d2) - (dn * dn));
    V Pm0 = mk(P2P2.x * -1.0, P2P2.y * -1.0, P2P2.z * -1.0);
    V v2 = sub(p, ld3(w[0]));
    double dot20 = dot(v2, P2P0), dot21 = dot(v2, Pm0);
    double cu = ((d2 * dot20) - (dn * dot21)) * bary, cv = ((d0 * dot21) - (dn * dot20)) * bary, cw = 1 - cu - cv;
    double uu = wu[0][0] * cw + wu[1][0] * cu + wu[2][0] * cv, vv = wu[0][1] * cw + wu[1][1] * cu + wu[2][1] * cv;
    u = uu * (T.w - 1);
    v = (1 - vv) * (T.h - 1);
  }
  if (CNT) ct.c[C_TEXEL]++;
  int ui = jd2i(u), vi = jd2i(v);
  long i00 = (long)vi * T.w + ui, i10 = i00 + T.w, i01 = i00 + 1, i11 = i10 + 1;
  V c00 = texel(S, T, i00), c10 = texel(S, T, i10), c01 = texel(S, T, i01), c11 = texel(S, T, i11);
  double fu = u - ui, fv = v - vi;
  V c0 = lerpc(c00, fu, c01), c1 = lerpc(c10, fu, c11);
  return lerpc(c0, fv, c1);
}

// myNoiseTexture.getClrAra (myTextureHandler.java:277-294): colours 0 and 1 interpolated by
// distVal, each channel scaled by float noise of the permuted, colorScale-scaled point
DEVI V clr_ara(const MatD& m, double distVal, V raw, int i0 = 0, int i1 = 1) {
  V pt = mk(raw.x * m.colorScale, raw.y * m.colorScale, raw.z * m.colorScale);
  double rm0 = 1.0, rm1 = 1.0, rm2 = 1.0;
  if (m.rndColors) {
    rm0 = 1.0 + (m.colorMult * noise3((float)pt.x, (float)pt.z, (float)pt.y));
    rm1 = 1.0 + (m.colorMult * noise3((float)pt.y, (float)pt.x, (float)pt.z));
    rm2 = 1.0 + (m.colorMult * noise3((float)pt.z, (float)pt.y, (float)pt.x));
  }
  const double* c0 = m.colors[i0];
  const double* c1 = m.colors[i1];
  return mk(jmax(0, jmin(1.0, (c0[0]) + rm0 * distVal * ((c1[0]) - (c0[0])))),
            jmax(0, jmin(1.0, (c0[1]) + rm1 * distVal * ((c1[1]) - (c0[1])))),
            jmax(0, jmin(1.0, (c0[2]) + rm2 * distVal * ((c1[2]) - (c0[2])))));
}

// java.util.Random as myCellularTexture uses it (new Random(hashInts(cell)), nextDouble)
struct JRand {
  uint64_t sd;
  DEVI void seed(int32_t s) { sd = ((uint64_t)(int64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
  DEVI int32_t next(int bits) {
    sd = (sd * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(int64_t)(sd >> (48 - bits));
  }
  DEVI double next_double() {
    const int64_t hi = next(26);
    return (double)((hi << 27) + next(27)) * 0x1.0p-53;
  }
};
DEVI int32_t fastfloor(double x) { return x > 0 ? jd2i(x) : jd2i(x) - 1; }  // DistRayTracer.java:307
DEVI int32_t hash_ints(int32_t x, int32_t y, int32_t z) {                    // DistRayTracer.hashInts (wraps)
  return (int32_t)((uint32_t)x * 1572869u + (uint32_t)y * 6291469u + (uint32_t)z);
}
// myCellularTexture.getDiffTxtrColor (myTextureHandler.java:433-480): Worley points of the
// 27 cells around the scaled hit (per-cell java.util.Random), the ROI function of the
// smallest distinct distances, mortar below the threshold, else a brick colour pair drawn
// from the nearest point's cell. The reference keeps every distance in a sorted map
// (an equal distance replaces the cell); only the numPtsDist (<= 8) smallest are read, so
// a sorted register list of 8 distinct distances gives the same keys and nearest cell.
DEVI V cellular_color(const MatD& m, const HitRec& h) {
  V hv = m.useFwdTrans ? h.fwd : h.hitLoc;
  hv = mk(hv.x * m.scale, hv.y * m.scale, hv.z * m.scale);
  const int32_t ix = fastfloor(hv.x), iy = fastfloor(hv.y), iz = fastfloor(hv.z);
  constexpr int KD = 8;
  double kd[KD];
  int32_t kn[KD];
#pragma unroll
  for (int i = 0; i < KD; ++i) { kd[i] = INFINITY; kn[i] = 0; }
  JRand rnd;
  for (int n = 0; n < 27; ++n) {  // DistRayTracer.nghbrHdCells order (:21-25): x-major over {0,1,-1}
    const int dx = (n / 9 == 2) ? -1 : n / 9, dy = ((n / 3) % 3 == 2) ? -1 : (n / 3) % 3, dz = (n % 3 == 2) ? -1 : n % 3;
    const int32_t cx = ix + dx, cy = iy + dy, cz = iz + dz;
    rnd.seed(hash_ints(cx, cy, cz));
    const double prob = rnd.next_double();
    int np = m.pdfVal[0];  // lowerKey(prob) (greatest key < prob), first entry when there is none
    for (int j = 1; j < m.npdf; ++j)
      if (m.pdfKey[j] < prob) np = m.pdfVal[j];
    for (int j = 0; j < np; ++j) {
      const double px = cx + rnd.next_double(), py = cy + rnd.next_double(), pz = cz + rnd.next_double();
      const double d = (m.distFunc == 0)
                           ? fabs(hv.x - px) + fabs(hv.y - py) + fabs(hv.z - pz)  // _L1Dist
                           : sqrt(((hv.x - px) * (hv.x - px)) + ((hv.y - py) * (hv.y - py)) + ((hv.z - pz) * (hv.z - pz)));
      bool eq = false;
#pragma unroll
      for (int i = 0; i < KD; ++i)
        if (kd[i] == d) { kn[i] = n; eq = true; }
      if (!eq && d < kd[KD - 1]) {  // sorted insert
#pragma unroll
        for (int i = KD - 1; i > 0; --i) {
          if (kd[i - 1] > d) { kd[i] = kd[i - 1]; kn[i] = kn[i - 1]; }
          else if (kd[i] > d) { kd[i] = d; kn[i] = n; }
        }
        if (kd[0] > d) { kd[0] = d; kn[0] = n; }
      }
    }
  }
  // myROI.calcROI variants (myTextureHandler.java:515-690) over the ascending distinct distances
  double dist = 0;
  int i = 0;
  double mod = -1;
#pragma unroll
  for (int q = 0; q < KD; ++q) {
    if (kd[q] == INFINITY) break;
    const double k = kd[q];
    switch (m.roiFunc) {
      case 0: dist += k; i++; break;                        // nearestROI
      case 2: dist += 1.0 / (mod * k); i++; break;          // altInvLinROI
      case 3: dist += (mod * pow(k, (double)(++i))); break;  // altExpROI
      case 4: dist += (mod * log(1 + k)); i++; break;       // altLogROI
      case 5: dist += pow(k, (double)(++i)); break;          // linExpROI
      case 6: dist += log(1 + k); i++; break;               // linLogROI
      case 7: dist += pow(k, (double)-(++i)); break;         // invExpROI
      case 8: dist += 1.0 / log(1 + k); i++; break;         // invLogROI
      default: dist += (mod * k); i++; break;               // altLinROI (1 and unknown)
    }
    if (i >= m.numPtsDist) break;
    mod *= -1;
  }
  if (m.roiFunc != 6) {  // fixDist (linLogROI returns its sum unfixed)
    if (dist < 0) dist *= -1;
    if (dist > 1.0) dist = 1.0 / dist;
  }
  dist = (dist < 0 ? 0 : dist > 1 ? 1 : dist);
  int brick = 0;
  if (!(dist < m.mortar)) {
    const int nb = kn[0];
    const int dx = (nb / 9 == 2) ? -1 : nb / 9, dy = ((nb / 3) % 3 == 2) ? -1 : (nb / 3) % 3, dz = (nb % 3 == 2) ? -1 : nb % 3;
    rnd.seed(hash_ints(ix + dx, iy + dy, iz + dz));
    const double res = rnd.next_double();
    brick = 2 * (1 + fastfloor(((m.ncolors / 2) - 1) * res));
  }
  return clr_ara(m, .65, hv, brick, brick + 1);
}

// getDiffTxtrColor of the shader's texture handler (myTextureHandler.java)
template <bool CNT, uint32_t F>
DEVI V diff_color(const SceneD& S, const MatD& m, const HitRec& h, const Key& k, double diffConst, Counters& ct) {
#ifdef RT_PROF_NOTEX  // profiling builds only (tools/variant_sweep.py): results differ
  if constexpr (false) {
#else
  if constexpr ((F & FT_TEX) != 0) {
#endif
    if (m.tex == 1) {  // myImageTexture :105-117
      V c = (m.texTop >= 0) ? image_color<CNT>(S, h, k, S.tex[m.texTop], ct) : ld3(m.diffuse);
      return mk(c.x * diffConst, c.y * diffConst, c.z * diffConst);
    }
    if ((F & FT_CELL) && m.tex == 5) {
      V out = cellular_color(m, h);
      if (fabs(diffConst - 1.0) > EPS) out = mk(out.x * diffConst, out.y * diffConst, out.z * diffConst);
      return out;
    }
    if (m.tex == 2 || m.tex == 3 || m.tex == 4 || m.tex == 6) {
      V hv = m.useFwdTrans ? h.fwd : h.hitLoc;
      hv = mk(hv.x * m.scale, hv.y * m.scale, hv.z * m.scale);  // getNoiseVal / getTurbVal scale hitVal in place
      V out;
      if (m.tex == 2) {  // myNoiseTexture :257-265
        double res = m.turbMult * noise3((float)hv.x, (float)hv.y, (float)hv.z);
        double val = .5 * res + .5;
        out = mk(val, val, val);
      } else if (m.tex == 4) {  // myMarbleTexture :366-377 with getAbsTurbVal :242-251
        double res = 0, fs = 1.0, as = 1.0;
        for (int i = 0; i < m.octaves; ++i) {
          res += fabs(noise3((float)(hv.x * fs), (float)(hv.y * fs), (float)(hv.z * fs))) * as;
          as *= .5;
          fs *= 1.92;
        }
        double lin = (hv.x * m.periodMult[0] + hv.y * m.periodMult[1] + hv.z * m.periodMult[2]);
        double spt = lin / m.pmMag + m.turbMult * res;
        double dv = .5 * jf::sin(spt) + .5;
        out = clr_ara(m, dv, hv);
      } else {  // wood: sqPtVal (myTextureHandler.java:275) + turbulence, banded by sin
        const double* pm = m.periodMult;
        double res;
        if (m.tex == 3) {  // myBaseWoodTexture :309-331: one noise octave
          res = noise3((float)hv.x, (float)hv.y, (float)hv.z);
        } else {  // myWoodTexture :334-356 with getTurbVal :225-233
          res = 0;
          double fs = 1.0, as = 1.0;
          for (int i = 0; i < m.octaves; ++i) {
            res += noise3((float)(hv.x * fs), (float)(hv.y * fs), (float)(hv.z * fs)) * as;
            as *= .5;
            fs *= 1.92;
          }
        }
        const double sq = sqrt((hv.x * hv.x) * pm[0] + (hv.y * hv.y) * pm[1] + (hv.z * hv.z) * pm[2]) + m.turbMult * res;
        double dv = jf::sin(sq * m.pmMag);
        if (m.tex == 3) {
          dv *= 1.1;
          dv += .5;
          dv = (dv < 0 ? 0 : (dv > 1 ? 1 : dv));
          out = clr_ara(m, dv, h.hitLoc);  // base wood: colours from the unscaled object-space hit
        } else {
          dv = 1 - (dv < 0 ? 0 : dv);
          out = clr_ara(m, dv, hv);
        }
      }
      if (fabs(diffConst - 1.0) > EPS) out = mk(out.x * diffConst, out.y * diffConst, out.z * diffConst);
      return out;
    }
  }
  return mk(m.diffuse[0] * diffConst, m.diffuse[1] * diffConst, m.diffuse[2] * diffConst);  // myNonTexture
}

// photon kNN gather: myKD_Tree.find_near / findNearbyNodes (myLight.java:389-445) and
// getIrradianceFromPhtnTree (myObjShader.java:441-458): the k nearest photons with
// d^2 < max_dist^2 (exact, shrinking radius), summed in the reference's poll order
// (farthest first) over pi * (largest d^2).
//
// Search: the photon BVH (csrc/photon.cpp), nearer child first, a child visited iff
// its box distance^2 < the current radius^2. The box distance is formed like the
// photon distance (per-axis differences, squares, same summation order) from bounds
// no closer than any photon inside, and IEEE rounding is monotonic, so it never
// exceeds the distance of a photon in the box: no qualifying photon is pruned.
// The max-heap of (d^2, photon) lives in scratch (one 16-byte entry per slot); it is
// filled by appending, heapified once when it first holds k entries, and afterwards
// updated by replacing the root -- the same k-set as push-then-poll.
static constexpr int KNN_MAX = 256;
struct KnnE {
  double d2;
  int32_t i, pad;
};
DEVI void knn_sift_down(KnnE* h, int n, int j) {
  const KnnE x = h[j];
  while (true) {
    int l = 2 * j + 1;
    if (l >= n) break;
    int m = l;
    if (l + 1 < n && h[l + 1].d2 > h[l].d2) m = l + 1;
    if (!(h[m].d2 > x.d2)) break;
    h[j] = h[m];
    j = m;
  }
  h[j] = x;
}
DEVI double box_d2(const double* mn, const double* mx, const double* p) {
  double d[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) d[c] = (p[c] < mn[c]) ? (p[c] - mn[c]) : ((p[c] > mx[c]) ? (p[c] - mx[c]) : 0.0);
  return d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
}
template <bool CNT>
DEVI V irradiance_heap(const SceneD& S, V p, Counters& ct) {
  if (S.nphoton == 0) return mk(0, 0, 0);
  KnnE hp[KNN_MAX];
  int hn = 0;
  const int K = S.photonK < KNN_MAX ? S.photonK : KNN_MAX;
  double maxd2 = S.photonMaxD2;
  const double pos[3] = {p.x, p.y, p.z};
  Stack st;  // (box d^2, node<<1 | side) ; the ray-traversal stack is idle during shading
  int sp = 0;
  int32_t N = S.photonRoot;
  while (true) {
    // N: a node to open
    const NodeD& nd = S.pnode[N];
    if (CNT) { ct.c[C_PHOTON]++; ct.c[C_WPHOTON]++; }
    const double dl = box_d2(nd.lmin, nd.lmax, pos), dr = box_d2(nd.rmin, nd.rmax, pos);
    const bool vl = dl < maxd2, vr = dr < maxd2;
    // the nearer child now, the other one pushed (re-checked against the radius when popped)
    int32_t next = -2;
    if (vl || vr) {
      const bool leftFirst = vl && (!vr || dl <= dr);
      const int side = leftFirst ? 0 : 1;
      if (vl && vr) { st.setT(sp, leftFirst ? dr : dl); st.setN(sp, (N << 1) | (1 - side)); sp++; }
      next = (N << 1) | side;
    }
    while (true) {
      if (next == -2) {  // pop
        if (sp == 0) break;
        --sp;
        if (!(st.getT(sp) < maxd2)) continue;
        next = st.getN(sp);
      }
      const NodeD& pn = S.pnode[next >> 1];
      const int side = next & 1;
      const int32_t child = side ? pn.right : pn.left;
      if (child >= 0) { N = child; break; }
      // leaf: scan its photons
      const int start = side ? pn.pad[2] : pn.pad[0], count = side ? pn.padR[0] : pn.pad[1];
      if (CNT) { ct.c[C_PHOTON] += count; ct.c[C_WPHOTON] += count; }
      for (int q = 0; q < count; ++q) {
        const double* ph = S.ppos + 3 * (size_t)(start + q);
        const double dx = pos[0] - ph[0], dy = pos[1] - ph[1], dz = pos[2] - ph[2];
        const double len2 = dx * dx + dy * dy + dz * dz;
        if (len2 < maxd2) {
          if (hn < K) {
            hp[hn].d2 = len2; hp[hn].i = start + q;
            hn++;
            if (hn == K) {  // heapify once, then the radius is the k-th distance
              for (int j = K / 2 - 1; j >= 0; --j) knn_sift_down(hp, K, j);
              if (hp[0].d2 < maxd2) maxd2 = hp[0].d2;
            }
          } else {  // len2 < maxd2 = root: replace the farthest
            hp[0].d2 = len2; hp[0].i = start + q;
            knn_sift_down(hp, K, 0);
            if (hp[0].d2 < maxd2) maxd2 = hp[0].d2;
          }
        }
      }
      next = -2;
    }
    if (next == -2 && sp == 0) {
      // finished (the inner loop broke out at an empty stack)
      break;
    }
  }
  if (hn == 0) return mk(0, 0, 0);  // [null] -> 0 (Q20)
  if (hn < K)
    for (int j = hn / 2 - 1; j >= 0; --j) knn_sift_down(hp, hn, j);
  const double rSq = hp[0].d2;
  const double area = PI_F * rSq;
  V res = mk(0, 0, 0);
  while (hn > 0) {  // poll order: farthest first
    const double* w = S.ppwr + 3 * (size_t)hp[0].i;
    res.x += w[0]; res.y += w[1]; res.z += w[2];
    hn--;
    hp[0] = hp[hn];
    knn_sift_down(hp, hn, 0);
  }
  return mk(res.x / area, res.y / area, res.z / area);
}

// Photon scan: f(d2, photon) for every photon with d2 < R2 (photon BVH, depth first,
// children pruned by box distance^2 >= R2; see box_d2). Order is irrelevant to its users.
template <bool CNT, bool PWR, int NL = STK_LDS, class Fn>
DEVI void photon_scan(const SceneD& S, const double* pos, double R2, Counters& ct, Fn&& f) {
  NStackT<NL> st;  // the ray-traversal stack is idle during shading
  int sp = 0;
  int32_t N = S.photonRoot;
  while (true) {
    const NodeD& nd = S.pnode[N];
    if (CNT) { ct.c[C_PHOTON]++; ct.c[C_WPHOTON]++; }
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const double* mn = side ? nd.rmin : nd.lmin;
      const double* mx = side ? nd.rmax : nd.lmax;
      if (!(box_d2(mn, mx, pos) < R2)) continue;
      const int32_t c = side ? nd.right : nd.left;
      if (c >= 0) { st.setN(sp++, c); continue; }
      const int start = side ? nd.pad[2] : nd.pad[0], count = side ? nd.padR[0] : nd.pad[1];
      if (CNT) { ct.c[C_PHOTON] += count; ct.c[C_WPHOTON] += count; }
      for (int q = 0; q < count; ++q) {
        const double* ph = S.ppos + 3 * (size_t)(start + q);
        const double dx = pos[0] - ph[0], dy = pos[1] - ph[1], dz = pos[2] - ph[2];
        const double d2 = dx * dx + dy * dy + dz * dz;  // myKD_Tree.find_near's distance, same order
        if (d2 < R2) {
          const double* pw = S.ppwr + 3 * (size_t)(start + q);
          f(d2, start + q, PWR ? mk(pw[0], pw[1], pw[2]) : mk(0, 0, 0));
        }
      }
    }
    if (sp == 0) break;
    N = st.getN(--sp);
  }
}

// photon_scan as a packet traversal (render kernel): the lanes shading nearby points of
// one pixel tile walk ONE photon-BVH node sequence -- the union of their own scans, in the
// same depth-first order (push left / right child, pop last-in first) -- with node
// records and leaf photons as scalar loads; a lane tests a child box, or a leaf's photons,
// only where its own scan would (lane mask per frame). Every lane therefore calls f with the
// same photons in the same order as photon_scan (results bit-identical) while each photon
// record is read once per wave instead of once per lane.
#ifndef RT_PH_BATCH
#define RT_PH_BATCH 1
#endif
static constexpr int PH_BATCH = RT_PH_BATCH;
#ifndef RT_PH_VLOAD
#define RT_PH_VLOAD 1
#endif
static constexpr int PH_VLOAD = RT_PH_VLOAD;  // leaf photons: vector load + v_readlane (0: scalar loads)
DEVI double rdlane(double v, int L) {  // lane L's v (wave-uniform result)
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, L);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), L);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// PWR: the photon's power goes to f too, loaded with its position (the photon is
// wave-uniform) instead of a dependent per-lane load inside f.
// Leaf photons (PH_VLOAD, default): the i-th lane running the scan loads the leaf's i-th
// photon (one coalesced vector load per leaf) and the photons are read back in leaf order
// with v_readlane; leaves with more photons than running lanes take the scalar loads.
template <bool CNT, bool PWR, class Fn>
DEVI void photon_scan_pk(const SceneD& S, const double* pos, double R2, Counters& ct, Fn&& f) {
  lds_i32* fN = pkN();  // the ray traversal's wave-uniform frames (idle during shading)
  lds_u64* fM = pkM();
  int sp = 0;
  int32_t N = S.photonRoot;
  const uint64_t act_all = __ballot(1);  // the lanes running this scan
  uint64_t act = act_all;
  while (true) {
    if (CNT && in_mask(act)) ct.c[C_PHOTON]++;
    WCNT(C_WPHOTON, 1);
    const NodeD* nd = S.pnode + N;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const ChildBox cb = sload_child(nd, side);
      bool in = false;
      if (in_mask(act)) in = box_d2(cb.mn, cb.mx, pos) < R2;
      const uint64_t m = __ballot(in);
      if (!m) continue;
      if (cb.ref >= 0) {
        fN[sp] = cb.ref;
        fM[sp] = m;
        sp++;
        continue;
      }
      const int start = sload(side ? &nd->pad[2] : &nd->pad[0]), count = sload(side ? &nd->padR[0] : &nd->pad[1]);
      if (CNT && in_mask(m)) ct.c[C_PHOTON] += count;
      WCNT(C_WPHOTON, count);
      if (PH_VLOAD && count <= __popcll(act_all)) {
        // the leaf's photons as ONE coalesced vector load (the i-th active lane loads photon i),
        // read back photon by photon with v_readlane: one memory round trip per leaf instead of
        // one scalar load batch per photon
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act_all >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act_all, 0u));
        double qx = 0, qy = 0, qz = 0;
        V qw = mk(0, 0, 0);
        if (rank < count) {
          const double* ph = S.ppos + 3 * (size_t)(start + rank);
          qx = ph[0]; qy = ph[1]; qz = ph[2];
          if (PWR) {
            const double* pp = S.ppwr + 3 * (size_t)(start + rank);
            qw = mk(pp[0], pp[1], pp[2]);
          }
        }
        uint64_t rem = act_all;  // lane of rank q: the q-th set bit
        for (int q0 = 0; q0 < count; q0 += PH_VLOAD) {  // PH_VLOAD independent distances per step
          double d2[PH_VLOAD];
          V pw[PH_VLOAD];
#pragma unroll
          for (int j = 0; j < PH_VLOAD; ++j) {
            const int L = (int)__builtin_ctzll(rem | (1ull << 63));  // past the leaf: any lane
            rem &= rem - 1;
            const double px = rdlane(qx, L), py = rdlane(qy, L), pz = rdlane(qz, L);
            pw[j] = PWR ? mk(rdlane(qw.x, L), rdlane(qw.y, L), rdlane(qw.z, L)) : mk(0, 0, 0);
            const double dx = pos[0] - px, dy = pos[1] - py, dz = pos[2] - pz;
            d2[j] = dx * dx + dy * dy + dz * dz;  // as photon_scan
          }
          if (in_mask(m)) {
#pragma unroll
            for (int j = 0; j < PH_VLOAD; ++j)
              if (q0 + j < count && d2[j] < R2) f(d2[j], start + q0 + j, pw[j]);
          }
        }
        continue;
      }
      for (int q0 = 0; q0 < count; q0 += PH_BATCH) {  // PH_BATCH photons' positions per scalar-load batch
        double px[PH_BATCH], py[PH_BATCH], pz[PH_BATCH];
        V pw[PH_BATCH];
#pragma unroll
        for (int j = 0; j < PH_BATCH; ++j)
          if (q0 + j < count) {
            const double* ph = S.ppos + 3 * (size_t)(start + q0 + j);
            px[j] = sload(ph); py[j] = sload(ph + 1); pz[j] = sload(ph + 2);
            if (PWR) {
              const double* pp = S.ppwr + 3 * (size_t)(start + q0 + j);
              pw[j] = mk(sload(pp), sload(pp + 1), sload(pp + 2));
            } else {
              pw[j] = mk(0, 0, 0);
            }
          }
#pragma unroll
        for (int j = 0; j < PH_BATCH; ++j)
          if (q0 + j < count && in_mask(m)) {
            const double dx = pos[0] - px[j], dy = pos[1] - py[j], dz = pos[2] - pz[j];
            const double d2 = dx * dx + dy * dy + dz * dz;  // as photon_scan
            if (d2 < R2) f(d2, start + q0 + j, pw[j]);
          }
      }
    }
    if (sp == 0) break;
    --sp;
    N = uni(fN[sp]);
    act = uni64(fM[sp]);
  }
}
// Divergent gathers scan lane by lane: when at least half of the lanes of a gather call (and at least
// two) lie farther than 2 start radii from the first lane's point -- the lanes of a pixel seen through
// the glass sphere, whose refracted samples spread over the floor -- each lane walks its own
// neighbourhood (photon_scan, stacks in scratch: the pkT levels hold the counting histogram) instead of
// one packet walking the union of all of them (those calls ran with ~6 lanes per wave step). Same
// photons in the same order per lane: the image is unchanged. C5 (t11): frame 195.2 -> 196.2 ms, but
// its slowest waves 47 -> 37 ms, the 8-GPU split's tail (profiles/r04f_*). RT_KNN_DIV = 0: packets only.
#ifndef RT_KNN_DIV
#define RT_KNN_DIV 1
#endif
#ifndef RT_KNN_DIV_FRAC
#define RT_KNN_DIV_FRAC 2
#endif
#ifndef RT_KNN_DIV_R
#define RT_KNN_DIV_R 2.0
#endif
template <bool CNT, bool PWR = false, class Fn>
DEVI void photon_scan_any(const SceneD& S, const double* pos, double R2, Counters& ct, Fn&& f, bool lanewise = false) {
  if (PACKET && RT_KNN_DIV > 0 && lanewise) photon_scan<CNT, PWR, 0>(S, pos, R2, ct, f);
  else if (PACKET) photon_scan_pk<CNT, PWR>(S, pos, R2, ct, f);
  else photon_scan<CNT, PWR>(S, pos, R2, ct, f);
}

// The k nearest photons by selection instead of a heap (no per-lane memory): the
// k-th smallest d^2 is bracketed by counting passes -- a histogram of equally spaced
// buckets of the current window [lo, hi): 64 u16 buckets in LDS (knn_hist_pass; KNN_EDGES
// = 16 u32 buckets when one lane has more than 65535 photons below hi, or 16 register
// counters in builds without the packet kernels) -- until the window holding the k-th
// photon has <= KNN_SHELL photons; a last pass sums every photon below the window and
// the nearest (k - below) window photons (kept sorted in registers). Same k-set and
// largest d^2 as the heap; the powers are summed in scan order rather than the
// reference's poll order (a last-ulp difference; DESIGN.md "Precision").
// Start window: [0, R2) with R2 from the local density of the smallest photon-BVH node
// around p holding >= k photons; if fewer than k photons fall below it, the next window starts
// there and extends by the density extrapolation, capped at that node's far-corner distance (all
// its photons lie within it), then max_dist^2.
#ifndef RT_KNN_SHELL
#define RT_KNN_SHELL 10
#endif
// A start window holding fewer than K photons (all of them in the set) is widened by the
// surface-density extrapolation of what is missing (count ~ d^2: hi x START x K / count), the new
// window starting above the counted photons, instead of straight to the enclosing node's far corner
// -- whose wide buckets then needed further passes. With that cheap recovery a tighter start window
// pays: C5 193.4 -> 179.1 ms at START 1.15 (1.0 / 1.1 / 1.2 / 1.25 / 1.3: 251 / 180.4 / 180.5 / 183.0 /
// 186.0 ms), the same k-sets and the same image bit for bit (profiles/r05j_*, r05k_*).
#ifndef RT_KNN_EXTRAP
#define RT_KNN_EXTRAP 1
#endif
#ifndef RT_KNN_START  // the start window: this many times the d^2 holding K photons at the node's density
#define RT_KNN_START 1.15
#endif
#ifndef RT_KNN_EDGES
#define RT_KNN_EDGES 16
#endif
#ifndef RT_KNN_LDS_HIST
#define RT_KNN_LDS_HIST 1
#endif
static constexpr int KNN_SHELL = RT_KNN_SHELL;
static constexpr int KNN_EDGES = RT_KNN_EDGES;  // counters per counting pass
// counting passes through a per-lane LDS histogram (packet kernels: the traversal stack's
// pkT levels are idle during shading) instead of KNN_EDGES register counters
static constexpr bool KNN_LDS_HIST = PACKET && RT_KNN_LDS_HIST != 0;
// KNN_H16: the LDS histogram as 64 u16 buckets (KNN_HB) instead of KNN_EDGES u32 ones
#ifndef RT_KNN_H16
#define RT_KNN_H16 1
#endif
static constexpr bool KNN_H16 = KNN_LDS_HIST && RT_KNN_H16 != 0;
// KNN_H8: 128 u8 buckets in the same words, so a pass narrows the window 8x further than 16 u32
// ones (a carry is detected by the buckets' sum; such a lane repeats the pass with the u16 buckets).
// Passes per gather call drop, C5 179.9 -> 175.0 ms, same image (profiles/r05n_c5_knn_h8_ab.log).
#ifndef RT_KNN_H8
#define RT_KNN_H8 1
#endif
static constexpr bool KNN_H8 = KNN_H16 && RT_KNN_H8 != 0;
static constexpr int KNN_HB = KNN_H8 ? 128 : KNN_H16 ? 64 : KNN_EDGES;
static_assert(!KNN_LDS_HIST || KNN_SHELL * 64 * 12 <= PK_LDS * 64 * 8, "window list fits the pkT levels");
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// One counting pass over [lo, hi) through a per-lane LDS histogram (packet kernels: the
// traversal stack's pkT levels are idle during shading) of NB equally spaced buckets:
// bucket j = #{k : e[k] <= d2} with e[k] = lo + (k + 1) w (k < NB - 1), e[NB - 1] = hi, and
// the counts c(k) = photons with d2 < e[k] (including those under lo) are its prefix sums.
// Yields c(NB - 1) (total) and the first edge kb with c(kb) >= K (-1: none), c(kb - 1) (0 for
// kb = 0) and c(kb). P16: two u16 buckets per LDS word (NB = 64 in the same 8 KB as 16 u32
// ones, so the first pass narrows 4x further); ovf reports more than 65535 photons below hi,
// whose counts may have carried between the halves (the caller repeats the pass with u32).
template <bool CNT, int NB, bool P16, bool P8 = false>
DEVI void knn_hist_pass(const SceneD& S, const double* pos, double lo, double hi, int K, Counters& ct,
                        uint32_t& total, int& kb, uint32_t& cPrev, uint32_t& cAt, bool& ovf, bool lw = false) {
  constexpr int NW = P8 ? NB / 4 : P16 ? NB / 2 : NB;  // LDS words per lane
  static_assert(NW * 64 * 4 <= PK_LDS * 64 * 8, "histogram fits the pkT levels");
  lds_u32* hist = (lds_u32*)pkT() + __lane_id();
#pragma unroll
  for (int q = 0; q < NW; ++q) hist[q * 64] = 0;
  uint32_t tot = 0;
  auto bump = [&](int j) {
    if (P8) {
      __hip_atomic_fetch_add(hist + (j >> 2) * 64, 1u << ((j & 3) * 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      tot++;
    } else if (P16) {
      __hip_atomic_fetch_add(hist + (j >> 1) * 64, 1u << ((j & 1) * 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      tot++;
    } else {
      __hip_atomic_fetch_add(hist + j * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  };
  const double w = (hi - lo) * (1.0 / NB);
  const double inv = NB / (hi - lo);
  // j0 from the scaled distance is biased low and raised by one exact edge compare, so j is
  // exact: the scaled distance and the edges carry rounding errors of ~4 NB hi / (hi - lo)
  // 2^-52 buckets, which the 2^-12 bias covers unless the window is 2^30 times narrower than hi
  const bool narrow = !((hi - lo) > hi * 0x1p-30);
  if (!__ballot(narrow)) {  // j0 is j or j - 1: one compare settles it (no loop)
    const double lob = lo + 0x1p-12 * w;  // the bias, as a shifted origin
    photon_scan_any<CNT>(S, pos, hi, ct, [&](double d2, int, V) {
      // j0 <= NB: d2 < hi; a j0 of NB (rounding) can only mean j = NB - 1, as the min keeps
      const int j0 = (int)fmax((d2 - lob) * inv, 0.0);
      bump(min(j0 + ((d2 < lo + (j0 + 1) * w) ? 0 : 1), NB - 1));  // e[j0] as below
    }, lw);
  } else {  // some lane's window is too narrow for the bias: walk the edges from 0
    photon_scan_any<CNT>(S, pos, hi, ct, [&](double d2, int, V) {
      int j = 0;
      while (j < NB - 1 && !(d2 < lo + (j + 1) * w)) ++j;
      bump(j);
    }, lw);
  }
  ovf = (P16 || P8) && tot > (uint32_t)S.knnU16Max;  // (the test knob lowers the u8 pass's limit too)
  uint32_t sum = 0;
  for (int q = 0; q < NW; ++q) {
    const uint32_t v = hist[q * 64];
#pragma unroll
    for (int h = 0; h < (P8 ? 4 : P16 ? 2 : 1); ++h) {
      const uint32_t c = P8 ? ((v >> (8 * h)) & 0xffu) : P16 ? ((v >> (16 * h)) & 0xffffu) : v;
      const uint32_t run = total + c;
      if (P8) sum += c;
      if (kb < 0 && (int)run >= K) { kb = P8 ? 4 * q + h : P16 ? 2 * q + h : q; cPrev = total; cAt = run; }
      total = run;
    }
  }
  if (P8 && sum != tot) ovf = true;  // a u8 carry: the buckets' sum falls short by 255 (256 out of a word)
}

// Exact replay of the reference's neighbourhood for ONE lane whose k-th distance is tied (several
// photons at the boundary distance, some in and some out): myKD_Tree.find_near (myLight.java:389-445)
// over the reference's own kd-tree (KdNodeD, built on the host like build_tree :332-381) with its
// java.util.PriorityQueue(reverseOrder) as JDK 8 sifts it -- an element moves up only past a strictly
// smaller parent and down only past a strictly larger child (the right child only when strictly
// larger than the left) -- so the photons evicted among equal distances are Java's; then
// getIrradianceFromPhtnTree (myObjShader.java:441-458): the powers summed in poll order (farthest
// first) over pi * (the first polled d2). The heap and the recursion's frames live in the wave's pkT
// LDS levels (idle once the counting selection's final pass is done); the lane runs alone.
// PriorityQueue.offer adds before poll trims: the heap holds K + 1 entries for a moment (K <= KNN_MAX)
static_assert((KNN_MAX + 1) * 12 + 64 * 4 <= PK_LDS * 64 * 8, "the replay's heap and frames fit the pkT levels");
#ifndef RT_KNN_JAVA_CALL  // the replay as a real call: the hot variants' register allocation stays as it was
#define RT_KNN_JAVA_CALL 1
#endif
#if RT_KNN_JAVA_CALL
#define KNN_JAVA_FN __device__ __attribute__((noinline))
#else
#define KNN_JAVA_FN DEVI
#endif
KNN_JAVA_FN V knn_java_(const NodeD* pnode, const double* ppos, const double* ppwr, int32_t root, int K, double maxd2,
                        double px, double py, double pz) {
  const double pos[3] = {px, py, pz};
  const int32_t off = pnode[root].padR[2];
  if (off <= 0) return mk(0, 0, 0);  // no kd-tree (unreachable: every photon map carries one)
  const KdNodeD* kd = reinterpret_cast<const KdNodeD*>(pnode + off);
  lds_f64* hd = pkT();                               // queue: d2 (K + 1 slots: offer, then poll)
  lds_i32* hx = (lds_i32*)(pkT() + KNN_MAX + 1);     // queue: photon (leaf order)
  lds_i32* stk = hx + KNN_MAX + 1;                   // frames: node << 2 | stage
  int n = 0;
  auto poll = [&]() {  // PriorityQueue.poll: the root goes, the last element sifts down from it
    --n;
    const double xd = hd[n];
    const int32_t xi = hx[n];
    if (n > 0) {
      int k = 0;
      const int half = n >> 1;
      while (k < half) {
        int c = 2 * k + 1;
        const int r = c + 1;
        if (r < n && hd[r] > hd[c]) c = r;
        if (xd >= hd[c]) break;
        hd[k] = hd[c]; hx[k] = hx[c];
        k = c;
      }
      hd[k] = xd; hx[k] = xi;
    }
  };
  int sp = 0;
  stk[sp++] = 0;  // the root (node 0), stage 0
  while (sp > 0) {
    const int32_t fr = stk[sp - 1];
    const int32_t node = fr >> 2;
    int stage = fr & 3;
    const KdNodeD kn = kd[node];
    const double* ph = ppos + 3 * (size_t)kn.photon;
    if (stage == 0) {
      if (kn.axis != -1) {  // the near side first (findNearbyNodes :411-423)
        const double delta = pos[kn.axis] - ph[kn.axis];
        const int32_t nearc = delta < 0 ? kn.left : kn.right;
        stk[sp - 1] = (node << 2) | 1;
        if (nearc != -1) { stk[sp++] = nearc << 2; continue; }
        stage = 1;
      } else {
        stage = 2;
      }
    }
    if (stage == 1) {  // the far side if the split plane is nearer than the current radius
      const double delta = pos[kn.axis] - ph[kn.axis], delta2 = delta * delta;
      const int32_t farc = delta < 0 ? kn.right : kn.left;
      stk[sp - 1] = (node << 2) | 2;
      if (farc != -1 && delta2 < maxd2) { stk[sp++] = farc << 2; continue; }
    }
    // the node's own photon (:425-444)
    const double dx = pos[0] - ph[0], dy = pos[1] - ph[1], dz = pos[2] - ph[2];
    const double len2 = dx * dx + dy * dy + dz * dz;
    if (len2 < maxd2) {
      int k = n++;  // PriorityQueue.offer: sift up
      while (k > 0) {
        const int parent = (k - 1) >> 1;
        if (hd[parent] >= len2) break;
        hd[k] = hd[parent]; hx[k] = hx[parent];
        k = parent;
      }
      hd[k] = len2; hx[k] = kn.photon;
      if (n > K) poll();
      if (n == K && hd[0] < maxd2) maxd2 = hd[0];
    }
    --sp;
  }
  if (n == 0) return mk(0, 0, 0);  // [null] -> 0 (Q20)
  const double area = PI_F * hd[0];
  V res = mk(0, 0, 0);
  while (n > 0) {  // poll order: farthest first
    const double* w = ppwr + 3 * (size_t)hx[0];
    res.x += w[0]; res.y += w[1]; res.z += w[2];
    poll();
  }
  return mk(res.x / area, res.y / area, res.z / area);
}
DEVI V knn_java(const SceneD& S, const double* pos) {
  return knn_java_(S.pnode, S.ppos, S.ppwr, S.photonRoot, S.photonK, S.photonMaxD2, pos[0], pos[1], pos[2]);
}

template <bool CNT>
DEVI V irradiance(const SceneD& S, V p, Counters& ct) {
#ifdef RT_KNN_HEAP
  return irradiance_heap<CNT>(S, p, ct);
#endif
  if (S.nphoton == 0) return mk(0, 0, 0);
  const int K = S.photonK;
  const double R2max = S.photonMaxD2;
  const double pos[3] = {p.x, p.y, p.z};
  // --- start bounds from the photon BVH: the smallest node containing p with >= K photons
  double R2far = R2max, R2dens = R2max;
  {
    int32_t N = S.photonRoot;
    while (true) {
      const NodeD& nd = S.pnode[N];
      int32_t nxt = -1;
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int32_t c = side ? nd.right : nd.left;
        const int cnt = side ? nd.padR[0] : nd.pad[1];
        const double* mn = side ? nd.rmin : nd.lmin;
        const double* mx = side ? nd.rmax : nd.lmax;
        if (c >= 0 && cnt >= K && nxt < 0 && box_d2(mn, mx, pos) == 0.0) nxt = c;
      }
      if (nxt < 0) {
        if (nd.padR[1] >= K) {
          double mn[3], mx[3], e[3], f[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            mn[c] = fmin(nd.lmin[c], nd.rmin[c]); mx[c] = fmax(nd.lmax[c], nd.rmax[c]);
            e[c] = mx[c] - mn[c];
            f[c] = fmax(pos[c] - mn[c], mx[c] - pos[c]);  // farthest corner, per axis
          }
          // every photon of the node is no farther than the far corner (monotonic rounding)
          const double far2 = (f[0] * f[0] + f[1] * f[1]) + f[2] * f[2];
          R2far = fmin(R2max, far2 * (1 + 0x1p-40));
          // photons lie on surfaces: density over the box's two largest extents
          const double a = fmax(fmax(e[0] * e[1], e[0] * e[2]), e[1] * e[2]);
          R2dens = fmin(R2far, RT_KNN_START * K * a / (PI_D * nd.padR[1]));
        }
        break;
      }
      N = nxt;
    }
  }
  bool lw = false;  // RT_KNN_DIV experiment: scan lane by lane
  if constexpr (PACKET && RT_KNN_DIV > 0) {
    const int f = (int)__builtin_ctzll(__ballot(1));
    const double fx = rdl(pos[0], f), fy = rdl(pos[1], f), fz = rdl(pos[2], f), r2 = rdl(R2dens, f);
    const double dx = pos[0] - fx, dy = pos[1] - fy, dz = pos[2] - fz;
    // RT_KNN_DIV = 1: 1 / RT_KNN_DIV_FRAC of the lanes in this call (at least two) are farther than
    // RT_KNN_DIV_R start radii; >= 2: at least that many lanes are
    const int nfar = __popcll(__ballot(!(dx * dx + dy * dy + dz * dz <= (RT_KNN_DIV_R * RT_KNN_DIV_R) * r2)));
    const int nact = __popcll(__ballot(1));
    lw = RT_KNN_DIV == 1 ? (nfar >= 2 && RT_KNN_DIV_FRAC * nfar >= nact) : nfar >= RT_KNN_DIV;
  }
  // --- bracket the k-th d^2: window [lo, hi), `below` photons under lo
  PROF_CNT(R_KNN_NCALL);
  double lo = 0, hi = R2dens;
  int below = 0;
  bool all = false;  // fewer than K photons within max_dist: the set is all of them
  for (int level = 0; level < 32; ++level) {
    PROF_T0(t_kc);
    constexpr int NE = KNN_EDGES;
    // c(k) = photons with d2 < e[k] (including the `below` ones); the pass yields c(NE - 1)
    // and the first edge kb with c(kb) >= K (-1: none), c(kb - 1) (0 for kb = 0) and c(kb)
    uint32_t total = 0, cPrev = 0, cAt = 0;
    int kb = -1;
    int ne = NE;  // this lane's edges in this pass: e[k] = lo + (k + 1) w, w = (hi - lo) / ne
    if constexpr (KNN_LDS_HIST) {
      bool ovf = false;
      knn_hist_pass<CNT, KNN_HB, KNN_H16 && !KNN_H8, KNN_H8>(S, pos, lo, hi, K, ct, total, kb, cPrev, cAt, ovf, lw);
      ne = KNN_HB;
      if (KNN_H8 && __ballot(ovf)) {  // a u8 bucket may have carried: this pass again with u16 buckets
        if (ovf) {
          total = cPrev = cAt = 0; kb = -1; ovf = false;
          knn_hist_pass<CNT, 64, true>(S, pos, lo, hi, K, ct, total, kb, cPrev, cAt, ovf, lw);
          ne = 64;
        }
      }
      if (KNN_H16 && __ballot(ovf)) {  // > 65535 photons below hi: this pass again with u32 buckets
        if (ovf) {
          total = cPrev = cAt = 0; kb = -1;
          knn_hist_pass<CNT, NE, false>(S, pos, lo, hi, K, ct, total, kb, cPrev, cAt, ovf, lw);
          ne = NE;
        }
      }
    } else {
      const double w = (hi - lo) * (1.0 / NE);
      double e[NE];
#pragma unroll
      for (int k = 0; k < NE - 1; ++k) e[k] = lo + (k + 1) * w;
      e[NE - 1] = hi;
      uint32_t c[NE];
#pragma unroll
      for (int k = 0; k < NE; ++k) c[k] = 0;
      photon_scan_any<CNT>(S, pos, hi, ct, [&](double d2, int, V) {
#pragma unroll
        for (int k = 0; k < NE; ++k) c[k] += (d2 < e[k]) ? 1u : 0u;
      });
      total = c[NE - 1];
#pragma unroll
      for (int k = 0; k < NE; ++k)  // selects, no dynamic register indexing
        if (kb < 0 && (int)c[k] >= K) { kb = k; cAt = c[k]; cPrev = k ? c[k - 1] : 0; }
    }
    PROF_ADD(t_kc, R_KNN_COUNT);
    PROF_CNT(R_KNN_NPASS);
    if ((int)total < K) {  // only possible for the start window: widen it
      if (hi == R2max) { all = true; break; }
#if RT_KNN_EXTRAP
      // every photon under hi is in the set: the window moves above it, and grows by the
      // surface-density extrapolation (count ~ d^2) of what is still missing, at most to R2far
      const double ext = total > 0 ? hi * (RT_KNN_START * K / (double)total) : R2far;
      lo = hi;
      below = (int)total;
      hi = (hi < R2far) ? fmin(R2far, ext) : R2max;
#else
      hi = (hi < R2far) ? R2far : R2max;
#endif
      continue;
    }
    // the window becomes [e[kb - 1], e[kb]) with e[k] = lo + (k + 1) w, e[ne - 1] = hi (the
    // pass's w: (hi - lo) / ne, an exact power-of-two scaling either way)
    const double wp = (hi - lo) * (ne == NE ? 1.0 / NE : ne == 64 ? 1.0 / 64 : 1.0 / 128);
    const double nhi = (kb == ne - 1) ? hi : lo + (kb + 1) * wp;
    const double nlo = kb ? lo + kb * wp : lo;
    const int nbelow = kb ? (int)cPrev : below, cb = (int)cAt;
    lo = nlo; hi = nhi; below = nbelow;
    if (cb - below <= KNN_SHELL || !(lo < hi)) break;
  }
  // --- final pass: every photon below the window, and the nearest K - below window photons
  PROF_T0(t_kf);
  double sd[KNN_SHELL];
  int32_t si[KNN_SHELL];
#pragma unroll
  for (int k = 0; k < KNN_SHELL; ++k) { sd[k] = DMAX; si[k] = -1; }
  V res = mk(0, 0, 0);
  double rSq = 0;
  int n = 0;
  int m = 0;  // window photons
  // window photon: keep the KNN_SHELL nearest, sorted (scan order breaks ties)
  auto shell_insert = [&](double xd, int32_t xi) {
#pragma unroll
    for (int k = 0; k < KNN_SHELL; ++k) {
      if (xd < sd[k]) {
        const double td = sd[k]; const int32_t ti = si[k];
        sd[k] = xd; si[k] = xi;
        xd = td; xi = ti;
      }
    }
  };
  if constexpr (KNN_LDS_HIST) {
    // window photons are appended to a per-lane list in LDS during the scan and sorted once
    // after it by the same insertion, in the same (scan) order. The window holds <= KNN_SHELL
    // photons unless the bracket ran out of levels, which only a window of equal distances
    // does: the list then keeps the first KNN_SHELL, as the sorted shell would.
    lds_f64* ld = pkT() + __lane_id();
    lds_i32* li = (lds_i32*)(pkT() + KNN_SHELL * 64) + __lane_id();
    photon_scan_any<CNT, true>(S, pos, all ? R2max : hi, ct, [&](double d2, int i, V w) {
      if (all || d2 < lo) {
        res.x += w.x; res.y += w.y; res.z += w.z;
        if (d2 > rSq) rSq = d2;
        n++;
      } else {
        if (m < KNN_SHELL) { ld[m * 64] = d2; li[m * 64] = i; }
        m++;
      }
    }, lw);
#pragma unroll
    for (int k = 0; k < KNN_SHELL; ++k)
      if (k < m) shell_insert(ld[k * 64], li[k * 64]);
  } else {
    photon_scan_any<CNT, true>(S, pos, all ? R2max : hi, ct, [&](double d2, int i, V w) {
      if (all || d2 < lo) {
        res.x += w.x; res.y += w.y; res.z += w.z;
        if (d2 > rSq) rSq = d2;
        n++;
      } else {
        shell_insert(d2, i);
        m++;
      }
    });
  }
  // a tie across the k-th position: window photons `need` and `need + 1` (1-based) at the same
  // distance. Which of them the reference keeps is its kd-tree order and heap layout: such a lane
  // replays find_near.
  bool tie = false;
  if (!all) {
    const int need = K - below;
    double dLast = -1, dNext = -2;
#pragma unroll
    for (int k = 0; k < KNN_SHELL; ++k) {
      if (k < need && si[k] >= 0) {
        const double* w = S.ppwr + 3 * (size_t)si[k];
        res.x += w[0]; res.y += w[1]; res.z += w[2];
        rSq = sd[k];
        n++;
      }
      if (k == need - 1) dLast = sd[k];
      if (k == need) dNext = sd[k];
    }
    // (a window of more photons than the shell holds -- only photons at one distance end the bracket
    // that way -- is replayed whether or not the tie straddles: the shell kept only its first ones)
    tie = need >= 1 && (m > KNN_SHELL || (need < m && dLast == dNext));
  }
  PROF_ADD(t_kf, R_KNN_FINAL);
  V out = mk(0, 0, 0);
  if (n > 0) {
    const double area = PI_F * rSq;
    out = mk(res.x / area, res.y / area, res.z / area);
  }
  for (uint64_t tl = __ballot(tie); tl; tl &= tl - 1)  // the tied lanes, one at a time
    if (__lane_id() == (unsigned)__builtin_ctzll(tl)) out = knn_java(S, pos);
  return out;
}

// skydome background (myScene.java:1104-1149)
template <bool CNT, uint32_t F>
DEVI V background(const SceneD& S, const WRay& w, Counters& ct) {
  if constexpr ((F & FT_TEX) != 0) {
    if (S.bkgTex >= 0) {
      const TexD& T = S.tex[S.bkgTex];
      double r = S.sky[0];
      V c = mk(S.sky[1], S.sky[2], S.sky[3]);
      V d = w.d, o = w.o;
      double a = ((d.x / r) * (d.x / r)) + ((d.y / r) * (d.y / r)) + ((d.z / r) * (d.z / r));
      V pC = mk((o.x - c.x) / r, (o.y - c.y) / r, (o.z - c.z) / r);
      double b = 2 * (((d.x / r) * pC.x) + ((d.y / r) * pC.y) + ((d.z / r) * pC.z));
      double cc = (pC.x * pC.x) + (pC.y * pC.y) + (pC.z * pC.z) - 1;
      double discr = ((b * b) - (4 * a * cc));
      double t = -DMAX;
      if (discr > 0) {
        double d1 = sqrt(discr), t1 = (-1 * b + d1) / (2 * a), t2 = (-1 * b - d1) / (2 * a), tv = jmin(t1, t2);
        if (tv < EPS) tv = jmax(t1, t2);
        t = tv;
      }
      V p = mk(d.x * t + o.x, d.y * t + o.y, d.z * t + o.z);
      double a0 = p.y - c.y, a1 = a0 / r;
      a1 = (a1 > 1) ? 1 : (a1 < -1) ? -1 : a1;
      double v = (T.h - 1) * jf::acos(a1) / PI_D;
      double shWm1 = T.w - 1, z1 = (p.z - c.z), q = v / (T.h - 1);
      double b0 = (p.x - c.x) / r;
      b0 = (b0 > 1) ? 1 : (b0 < -1) ? -1 : b0;
      double b1 = jf::sin(q * PI_D);
      double a2 = (fabs(b1) < EPS) ? 1 : b0 / b1;
      double u = (z1 <= EPS) ? ((shWm1 * (jf::acos(a2)) / (TWO_PI_F)) + shWm1 / 2.0) : shWm1 - ((shWm1 * (jf::acos(a2)) / (TWO_PI_F)) + shWm1 / 2.0);
      u = (u < 0) ? 0 : (u > shWm1) ? shWm1 : u;
      if (CNT) ct.c[C_TEXEL]++;
      return texel(S, T, (long)jd2i(v) * T.w + jd2i(u));
    }
  }
  return mk(uni_here(S.bg[0]), uni_here(S.bg[1]), uni_here(S.bg[2]));
}

DEVI V rot_axis(V v1, V u, double thet) {  // rotVecAroundAxis (DistRayTracer.java:336-349)
  double cT = jf::cos(thet), sT = jf::sin(thet), oneMC = 1 - cT, ux2 = u.x * u.x, uy2 = u.y * u.y, uz2 = u.z * u.z,
         uxy = u.x * u.y, uxz = u.x * u.z, uyz = u.y * u.z, uzS = u.z * sT, uyS = u.y * sT, uxS = u.x * sT,
         uxzC1 = uxz * oneMC, uxyC1 = uxy * oneMC, uyzC1 = uyz * oneMC;
  return mk((ux2 * oneMC + cT) * v1.x + (uxyC1 - uzS) * v1.y + (uxzC1 + uyS) * v1.z,
            (uxyC1 + uzS) * v1.x + (uy2 * oneMC + cT) * v1.y + (uyzC1 - uxS) * v1.z,
            (uxzC1 - uyS) * v1.x + (uyzC1 + uxS) * v1.y + (uz2 * oneMC + cT) * v1.z);
}
// U: L is wave-uniform (light_sum's loop): its fields as scalar loads
template <bool U = false>
DEVI V disk_pos(const LightD& L, const Key& k, uint32_t kk) {  // getRandomDiskPos (myLight.java:251-258)
  const int32_t li = pld<U>(&L.index);
  double th = rng(k.seed, k.pixel, k.sample, k.node, SITE_DISK + li, kk, 0, TWO_PI_F);
  V r = nrmz(rot_axis(pld3<U>(L.tangent), pld3<U>(L.orient), th));
  double m = rng(k.seed, k.pixel, k.sample, k.node, SITE_DISK + li, kk + 1, 0, pld<U>(&L.radius));
  r = mk(r.x * m, r.y * m, r.z * m);
  return mk(r.x + pld<U>(L.origin), r.y + pld<U>(L.origin + 1), r.z + pld<U>(L.origin + 2));
}

// calcShadowColor (myObjShader.java:98-153)
// pow for shading terms: integer exponents 0..1024 by binary exponentiation (within ~20
// ulps of pow for the phong exponents used; ocml's double pow is ~40x the instructions)
// the general pow as a real call: inlined, its polynomial constants are hoisted to the kernel
// entry (loop-invariant VGPRs), spilled, and cost every wave a scratch round trip although
// integer exponents never reach it
__device__ __attribute__((noinline)) double pow_call(double x, double e) { return pow(x, e); }
DEVI double pow_shade(double x, double e) {
  if (!(e >= 0 && e <= 1024 && e == floor(e))) return pow_call(x, e);
  int n = (int)e;
  double r = 1, b = x;
  while (n) {
    if (n & 1) r *= b;
    n >>= 1;
    if (n) b *= b;
  }
  return r;
}
// STASH (packet kernels): h.nrm, h.dw and tex are in the LDS slots (shade_node), the sums too
template <bool CNT, uint32_t F, bool STASH>
DEVI V light_sum(const SceneD& S, const MatD& m, const HitRec& h, V tex, const Key& k, Counters& ct) {
  double r = 0, g = 0, b = 0;
  if (STASH) stash3(SL_RGB, mk(0, 0, 0));
  if constexpr (WAVE_CULL<F>) {
    if (S.fastSlab & SCENE_WAVE_CULL) step_cands(S, h.fwd);
    else step_cands_all();
  }
  for (int li = 0; li < S.nlight; ++li) {
    if (STASH) lds_barrier();
    const LightD& L = S.light[li];
    // li is wave-uniform: the light record's hot fields are scalar loads
    const int32_t ltype = sload(&L.type);
    double lg[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) lg[q] = sload(L.g + q);
    const V lorg = mk(sload(L.origin), sload(L.origin + 1), sload(L.origin + 2));
    const V lcol = mk(sload(L.color), sload(L.color + 1), sload(L.color + 2));
    const bool disk = (F & FT_LIGHTX) && ltype == 2;
    V lo = disk ? disk_pos<(RT_ULOAD & 2) != 0>(L, k, 0) : lorg;
    V ln = xpt(lg, lo);
    ln = nrmz(mk(ln.x - h.fwd.x, ln.y - h.fwd.y, ln.z - h.fwd.z));
    WRay sr;
    sr.o = h.fwd;
    sr.d = nrmz(ln);  // myRay ctor normalises again
    sr.d0 = sr.d;
    sr.stable = false;
    sr.moved = false;
    sr.ver = 0;
    V lo2 = disk ? disk_pos<(RT_ULOAD & 2) != 0>(L, k, 2) : lorg;
    double t = sqrt((((sr.o.x - lo2.x) * (sr.o.x - lo2.x)) + ((sr.o.y - lo2.y) * (sr.o.y - lo2.y))) + ((sr.o.z - lo2.z) * (sr.o.z - lo2.z)));
    double ltMult = 1;
    if (CNT) ct.c[C_LIGHT]++;
    WCNT(C_WLIGHT, 1);  // the light record: scalar loads, once per wave
    if ((F & FT_LIGHTX) && ltype == 1) {  // mySpotLight.intersectCheck / calcT_Mult (myLight.java:77-82,159-163)
      constexpr bool U = (RT_ULOAD & 2) != 0;
      double angle = jf::acos(-1 * dot(sr.d, pld3<U>(L.orient)));
      const double inR = pld<U>(&L.innerRad), outR = pld<U>(&L.outerRad);
      ltMult = (angle < inR) ? 1 : (angle > outR) ? 0 : (outR - angle) / pld<U>(&L.radDiff);
    }
    if (ltMult == 0) continue;
    if (CNT) ct.c[C_SHADOW]++;
    Key sk = k;
    sk.tsite = SITE_SHADOW_TIME + li;
    PKSTAT(P_SH_STEP, __ballot(1));
    if (STASH && (F & FT_LIGHTX)) { stash(SL_LTM, ltMult); lds_barrier(); }
#ifdef RT_PROF_NOSHADOW  // profiling builds only (tools/variant_sweep.py): results differ
    if (false)
#endif
    if (shadowed<CNT, F, PACKET, WAVE_CULL<F>>(S, sr, sk, t, ct, li)) continue;
    renorm(sr);  // shadowRay.direction._normalize()
    if (STASH) {
      if (F & FT_LIGHTX) ltMult = unstash(SL_LTM);
      const V rgb = unstash3(SL_RGB);
      r = rgb.x; g = rgb.y; b = rgb.z;
    }
    const V hn = STASH ? unstash3(SL_NRM) : h.nrm;
    double ldp = dot(sr.d, hn) * ltMult;
    if (ldp > EPS) {
      const V tx = STASH ? unstash3(SL_TEX) : tex;
      r += tx.x * lcol.x * ldp;
      g += tx.y * lcol.y * ldp;
      b += tx.z * lcol.z * ldp;
    }
    if (STASH) stash3(SL_RGB, mk(r, g, b));
#ifdef RT_PROF_NOPHONG  // profiling builds only: results differ
    continue;
#endif
    if (m.phong == 0) continue;
    // the specular term only adds colour (no hit / shadow / branch decision depends on it):
    // it is evaluated to a few ulps instead of the reference's exact operation order --
    // H normalised with one reciprocal, integer phong exponents by squaring
    const V hdw = STASH ? unstash3(SL_DW) : h.dw;
    const V hv = mk(sr.d.x - hdw.x, sr.d.y - hdw.y, sr.d.z - hdw.z);
    const double hm = mag(hv), hr = hm == 0 ? 1.0 : 1.0 / hm;
    double hdp = (hv.x * hr * hn.x + hv.y * hr * hn.y + hv.z * hr * hn.z) * ltMult;
    if (hdp > EPS) {
      double ph = pow_shade(hdp * hdp, m.phong);
      r += m.specular[0] * lcol.x * ph;
      g += m.specular[1] * lcol.y * ph;
      b += m.specular[2] * lcol.z * ph;
      if (STASH) stash3(SL_RGB, mk(r, g, b));
    }
  }
  if (STASH) { lds_barrier(); return unstash3(SL_RGB); }
  return mk(r, g, b);
}

DEVI V refl_dir(V eye, V n) {  // compReflDir (myObjShader.java:89-96)
  double dp = 2 * dot(eye, n);
  V tv = mk(n.x * dp, n.y * dp, n.z * dp);
  return nrmz(sub(tv, eye));
}

// Fresnel split shared by calcTransClr (myObjShader.java:157-276), calcTransRay
// (:297-397, photons) and the simple shader's calcSimpleTransClr (:503-631).
struct TransOut {
  V refr, refl;  // refraction dir; reflection dir (already x refractNormMult)
  double omtr, tr;
  bool doA, doB;
};
DEVI TransOut trans_split(const MatD& m, const HitRec& h, const double* inKt, bool strans) {
  TransOut T;
  V back = mk(h.dw.x * -1, h.dw.y * -1, h.dw.z * -1);
  V N = h.nrm;
  double cos1 = dot(back, N), rnm = 1.0;
  if (cos1 < EPS) { rnm = -1.0; N = mk(N.x * -1, N.y * -1, N.z * -1); }
  cos1 = dot(back, N);
  double mb = mag(back), mn = mag(N);
  double thetaI = jf::acos(dot(back, N) / (mb * mn));  // _angleBetween (DistRayTracer.java:445-452)
  double idx = strans ? m.perm : m.ktrans;
  double n = 1, n1 = 0, n2 = 0, cos2 = 0, tr = 0, omtr = 1;
  bool TIR = false;
  if (rnm < 0) {  // leaving the material
    double thetaCrit = jf::asin(1.0 / idx);
    if (thetaI < thetaCrit) {
      n1 = idx; n2 = 1; n = (n1 / n2);
      cos2 = sqrt(1.0 - (n * n) * (1.0 - (cos1 * cos1)));
    } else {
      tr = 1; omtr = 1 - tr; TIR = true; cos2 = 0;
    }
  } else {
    n1 = strans ? inKt[1] : inKt[0];
    n2 = idx;
    n = (n1 / n2);
    cos2 = sqrt(1.0 - (n * n) * (1.0 - (cos1 * cos1)));
  }
  if (!TIR) {  // Fresnel with cos(theta_t) = sqrt(1 - (n1/n2) sin^2) (Q15)
    double sa = jf::sin(jf::acos(cos1)), rct = sqrt(1.0 - ((n1 / n2) * sa * sa));
    double a1 = n1 * cos1, b1 = n2 * rct, nd1 = (a1 - b1) / (a1 + b1);
    double a2 = n1 * rct, b2 = n2 * cos1, nd2 = (a2 - b2) / (a2 + b2);
    tr = ((nd1 * nd1) + (nd2 * nd2)) / 2.0;
    omtr = 1 - tr;
  }
  T.omtr = omtr;
  T.tr = tr;
  T.doA = strans ? (omtr > 0) : (omtr > EPS);
  T.doB = strans ? (tr > 0) : (tr > EPS);
  V u = mk(back.x * (n * -1), back.y * (n * -1), back.z * (n * -1));
  double kk = (n * cos1) - cos2;
  V nv = mk(N.x * kk, N.y * kk, N.z * kk);
  T.refr = nrmz(mk(u.x + nv.x, u.y + nv.y, u.z + nv.z));
  V rd = refl_dir(back, N);
  T.refl = mk(rd.x * rnm, rd.y * rnm, rd.z * rnm);
  return T;
}

// ---------------------------------------------------------------------------
// shading tree. A node spawns child A at once; a frame keeps what the node
// needs when its children return: local colour, accumulated child sum,
// weights, and (two-child nodes only) the second child's ray.
//
// The ray's medium (myRay.currKTrans, myRay.java:26-47) is a material index: the reference
// copies {KTrans, perm, permClr} of the material that spawned a refracted ray, or all 1s
// (camera / reflected rays, the simple shader's reflection), and reads only entries 0 and 1
// (calcTransClr n1, myObjShader.java:193; calcSimpleTransClr :525).
struct Child {  // outgoing ray
  V o, d;
  int32_t ktm;  // medium: material whose (ktrans, perm) are currKTrans[0..1]; -1 = all 1s
  uint32_t node;
  int32_t gen;
};
DEVI void kt_of(const SceneD& S, int32_t ktm, double ik[2]) {
  if (ktm < 0) { ik[0] = 1; ik[1] = 1; }
  else { ik[0] = S.mat[ktm].ktrans; ik[1] = S.mat[ktm].perm; }
}
// Transparent variants: weights are rebuilt from the material at the child's return with
// the same products the reference forms (omtr * permClr, tr * kRefl, ...), so a frame holds
// two scalars instead of two colours; the B child's medium is the material again.
// Only the fields a node's case needs are written (the frame stack lives in scratch).
enum : uint8_t { FM_REFL = 0, FM_FRESNEL = 1, FM_SIMPLE = 2 };  // weight rule of a frame
// FRAME_SLIM (trace_sample's frames): the rule is rebuilt from the material, omtr from tr (trans_split
// forms omtr as 1 - tr on every path), the node id from the returning child's id and the generation
// from the stack index, so a Fresnel frame writes 24 B fewer to scratch. C4: writes 143.9 -> 127.0 GB
// per frame, 456.9 -> 453.8 ms; C5 174.3 -> 173.9 ms; same images (profiles/r05q_frame_slim_ab.log)
#ifndef RT_FRAME_SLIM
#define RT_FRAME_SLIM 1
#endif
static constexpr bool FRAME_SLIM = RT_FRAME_SLIM != 0;
template <uint32_t F>
struct FrameT {
  V local, acc, org, dB;  // acc: child A's weighted colour, kept only while B is traced
  double wa, wb;          // FM_FRESNEL / FM_SIMPLE: omtr, tr of the split
  int32_t mat;
  uint32_t node;
  int32_t gen;
  uint8_t phase, hasB, mode;  // phase 1: A out; 2: B out after A; 3: B out, no A
};
template <uint32_t F>
struct FrameR {  // no transparent materials: at most one child (reflection), weight = mat.kreflclr
  V local;
  int32_t mat;
  uint8_t phase;
};
template <uint32_t F>
using FrameOf = typename std::conditional<(F & FT_TRANS) != 0, FrameT<F>, FrameR<F>>::type;

// getColorAtPos (myObjShader.java:409-438; simple shader :635-651): local colour and the
// children. Returns the number of children (0..2); child A is written to `a`, the local colour to
// `loc` -- not to the frame: the caller stores it there only when the node pushes one (a node
// without children keeps it in registers; the frame stack lives in scratch).
template <bool CNT, uint32_t F, bool SLIM = FRAME_SLIM>  // SLIM: the frame's derivable fields are not written
DEVI int shade_node(const SceneD& S, const HitRec& h, const Child& in, const Key& k, FrameOf<F>& Fr, V& loc,
                    Child& a, bool& branch, Counters& ct) {
  const MatD& m = S.mat[h.mat];
  double r = m.ambient[0], g = m.ambient[1], b = m.ambient[2];
  if constexpr ((F & FT_PHOTON) != 0) {
    if (!m.simple && (m.krefl == 0.0) && m.usePhotonMap) {
#ifdef RT_PROF_NOGATHER  // profiling builds only: results differ
      V ir = mk(0, 0, 0);
#else
      PROF_T0(t_ph);
      V ir = irradiance<CNT>(S, h.fwd, ct);
      PROF_ADD(t_ph, R_PHOTON);
#endif
      if (m.isCausticPhtn) { r += ir.x; g += ir.y; b += ir.z; }
      else { r += m.diffuse[0] * ir.x; g += m.diffuse[1] * ir.y; b += m.diffuse[2] * ir.z; }
    }
  }
  PROF_T0(t_tex);
  V tex = diff_color<CNT, F>(S, m, h, k, m.simple ? 1.0 : m.diffConst, ct);
  PROF_ADD(t_tex, R_TEX);
  PROF_T0(t_ls);
  V ls;
  HitRec hs = h;  // the hit as the rest of the node sees it (STASH: normal / view direction from LDS)
  if constexpr (STASH_SHADE) {
    stash3(SL_BASE, mk(r, g, b)); stash3(SL_TEX, tex); stash3(SL_NRM, h.nrm); stash3(SL_DW, h.dw);
    lds_barrier();
    ls = light_sum<CNT, F, true>(S, m, h, tex, k, ct);
    lds_barrier();
    hs.nrm = unstash3(SL_NRM); hs.dw = unstash3(SL_DW);
    const V base = unstash3(SL_BASE);
    r = base.x; g = base.y; b = base.z;
  } else {
    ls = light_sum<CNT, F, false>(S, m, h, tex, k, ct);
  }
  PROF_ADD(t_ls, R_LIGHT);
  r += ls.x; g += ls.y; b += ls.z;
  loc = mk(r, g, b);
  branch = (in.gen < S.numRays - 2) && m.hasCaustic;
#ifdef RT_PROF_NOSECONDARY  // profiling builds only: results differ
  branch = false;
#endif
  if (!branch) return 0;
  a.o = h.fwd;
  if (STASH_SHADE) stash3(SL_RAYO, a.o);  // the child ray goes to trace_sample through LDS
  a.gen = in.gen + 1;
  a.node = in.node * 2;
  if constexpr ((F & FT_TRANS) != 0) {
    bool trans = !m.simple && ((m.ktrans > 0) || (m.perm > 0.0));
    bool strans = m.simple && (m.ktrans > 0);
    if (trans || strans) {  // calcTransClr :157-276 / calcSimpleTransClr :503-631
      double ik[2];
      kt_of(S, in.ktm, ik);
      const TransOut T = trans_split(m, hs, ik, strans);
      // children's medium: the material's {KTrans, perm, permClr}; the simple shader's
      // reflection child gets all 1s
      Fr.mat = h.mat;
      if (!SLIM) {
        Fr.mode = strans ? FM_SIMPLE : FM_FRESNEL;
        Fr.wa = T.omtr;
      }
      Fr.wb = T.tr;
      if (T.doA) {
        a.d = T.refr;
        if (STASH_SHADE) stash3(SL_RAYD, a.d);
        a.ktm = h.mat;
        if (CNT) ct.c[C_REFR]++;
        Fr.phase = 1;
        Fr.hasB = T.doB;
        if (T.doB) {
          Fr.dB = T.refl;
          Fr.org = h.fwd;
          if (!SLIM) {
            Fr.node = in.node;
            Fr.gen = in.gen;
          }
        }
        return T.doB ? 2 : 1;
      }
      if (T.doB) {  // only the reflection child: spawn it as "B"
        a.d = T.refl;
        if (STASH_SHADE) stash3(SL_RAYD, a.d);
        a.node = in.node * 2 + 1;
        a.ktm = strans ? -1 : h.mat;
        if (CNT) ct.c[C_REFL]++;
        Fr.phase = 3;
        return 1;
      }
      return 0;
    }
  }
  if (m.krefl > 0.0) {  // calcReflClr :278-294
    V back = mk(hs.dw.x * -1, hs.dw.y * -1, hs.dw.z * -1);
    V rd = refl_dir(back, hs.nrm);
    if (dot(rd, hs.nrm) >= 0) {
      a.d = rd;
      if (STASH_SHADE) stash3(SL_RAYD, a.d);
      a.ktm = -1;
      Fr.mat = h.mat;
      if constexpr ((F & FT_TRANS) != 0) {  // FrameR's fold reads only local and mat
        Fr.phase = 1;
        if (!SLIM) Fr.mode = FM_REFL;
        Fr.hasB = 0;
      }
      if (CNT) ct.c[C_REFL]++;
      return 1;
    }
  }
  return 0;
}

DEVI V clampc(V c) { return mk(jmin(1, c.x), jmin(1, c.y), jmin(1, c.z)); }  // myColor ctor

static constexpr int MAX_FRAMES = 7;  // gen < numRays-2 = 6 -> at most 6 nodes with children

// A lane whose shading tree is finished waits, with its colour, until the wave's last lane leaves
// the loop. Held in VGPRs, that colour is live across every later iteration of the other lanes'
// trees, and at 128 VGPRs the compiler spilled it to scratch and reloaded it on every iteration
// (C3: ~30 B of scratch writes per sample). It waits in the lane's own LDS stash slots instead:
// every LDS slot the other lanes write while tracing and shading is their own ([slot][lane]:
// traversal levels, stash slots), except the per-lane stacks of the photon scans and of the
// lane-wise BVH experiment (RT_LANE_DIV), which index [level][lane] ints over the same bytes -- so
// not in photon variants nor with RT_LANE_DIV. Measured (profiles/r04z_res_lds_ab.txt): C3 writes
// 1.36 -> 1.31 GB per frame at the same time; C4's transparent variant lost 1.8 % then (its allocation
// shifted) and gains since round 5 (below).
// Round 5, after the scalar primitive loads and slim frames shifted C4's allocation: the per-pixel
// sums and the finished colour in LDS pay in the transparent variants without a photon map too --
// C4 455.3 -> 447.4 ms, writes 127.0 -> 113.1 GB per frame; C5's photon variant keeps its sums in
// VGPRs (177.6 vs 174.4 ms with them in LDS), same images (profiles/r05z_trans_lds_ab.log)
#ifndef RT_RES_LDS_TRANS
#define RT_RES_LDS_TRANS 1
#endif
#ifndef RT_SUMS_LDS_TRANS
#define RT_SUMS_LDS_TRANS 1
#endif
#ifndef RT_RES_LDS
#define RT_RES_LDS 1
#endif
enum { SL_RES = SL_RGB };
template <uint32_t F>
static constexpr bool RES_LDS = RT_RES_LDS != 0 && STASH_SHADE && (F & FT_PHOTON) == 0 &&
                                ((F & FT_TRANS) == 0 || RT_RES_LDS_TRANS != 0) && RT_LANE_DIV == 0;

// reflectRay (myScene.java:907-914) for the whole shading tree of one camera sample
template <bool CNT, uint32_t F>
DEVI V trace_sample(const SceneD& S, V org, V dir, Key k, Counters& ct) {
  FrameOf<F> fr[MAX_FRAMES];
  int sp = 0;
  Child in;
  in.o = org; in.d = dir; in.node = 1; in.gen = 0; in.ktm = -1;
  // STASH_SHADE: the next ray of the tree waits in LDS (stash slots) across the loop's back edge
  if (STASH_SHADE) { stash3(SL_RAYO, in.o); stash3(SL_RAYD, in.d); }
  while (true) {
    V c;
    {
      if (STASH_SHADE) { lds_barrier(); in.o = unstash3(SL_RAYO); in.d = unstash3(SL_RAYD); }
      WRay w;
      w.o = in.o; w.d = nrmz(in.d); w.d0 = w.d; w.stable = false; w.moved = false; w.ver = 0;  // myRay ctor
      k.node = in.node;
#ifdef RT_PROF_NOTRACE  // profiling builds only (tools/variant_sweep.py): results differ
      Best b = miss();
#else
      PKSTAT(P_RAY_STEP, __ballot(1));
      Best b = closest<CNT, F, PACKET>(S, w, k, ct);
#endif
      if (b.t == DMAX) {
        PROF_T0(t_bg);
        c = background<CNT, F>(S, w, ct);
        if constexpr (RES_LDS<F>) { stash3(SL_RES, c); lds_barrier(); }
        PROF_ADD(t_bg, R_BG);
#ifdef RT_PROF_NOSHADE
      } else if (true) {
        c = mk(b.t * 0.01, 0, 0);
        if constexpr (RES_LDS<F>) { stash3(SL_RES, c); lds_barrier(); }
#endif
      } else {
        PROF_T0(t_hit);
        HitRec h = make_hit<F>(S, b, w, k);
        PROF_ADD(t_hit, R_HIT);
        bool branch;
        Child a;
        FrameOf<F>& Fr = fr[sp];
        V loc;
        PROF_T0(t_sh);
        int nch = shade_node<CNT, F>(S, h, in, k, Fr, loc, a, branch, ct);
        PROF_ADD(t_sh, R_SHADE);
        if (nch > 0 && sp < MAX_FRAMES) {
          Fr.local = loc;
          sp++;
          in = a;  // STASH_SHADE: its o / d are already in the LDS slots (shade_node)
          continue;
        }
        c = branch ? clampc(add(loc, mk(0, 0, 0))) : clampc(loc);  // no child: acc stayed 0
        if constexpr (RES_LDS<F>) { stash3(SL_RES, c); lds_barrier(); }
      }
    }
    if constexpr (RES_LDS<F>) {  // the ray's colour reaches the fold through the lane's LDS slots
      lds_barrier();
      c = unstash3(SL_RES);
    }
    // deliver finished colours upward
    bool spawned = false;
    uint32_t cn = in.node;  // FRAME_SLIM: the node id of the subtree that just finished
    while (sp > 0) {
      FrameOf<F>& P = fr[sp - 1];
      if constexpr ((F & FT_TRANS) == 0) {  // the only child has returned
        const double* wA = S.mat[P.mat].kreflclr;
        V acc = mk(0 + (wA[0] * c.x), 0 + (wA[1] * c.y), 0 + (wA[2] * c.z));
        c = clampc(add(P.local, acc));
        sp--;
      } else {
        // the weights of the reference's frame, rebuilt from the material (same products)
        const MatD& m = S.mat[P.mat];
        const uint8_t ph = P.phase;
        uint8_t mode;
        double wa;
        if (FRAME_SLIM) {  // the frame's rule from its material (shade_node's case split), omtr = 1 - tr
          const bool strans = m.simple && (m.ktrans > 0);
          const bool trans = !m.simple && ((m.ktrans > 0) || (m.perm > 0.0));
          mode = (trans || strans) ? (strans ? FM_SIMPLE : FM_FRESNEL) : FM_REFL;
          wa = 1 - P.wb;
        } else {
          mode = P.mode;
          wa = P.wa;
        }
        const uint32_t pn = cn >> 1;  // FRAME_SLIM: this frame's node id (its child's id / 2)
        cn = pn;
        V acc;
        if (ph == 1) {
          V wA;
          if (mode == FM_REFL) wA = mk(m.kreflclr[0], m.kreflclr[1], m.kreflclr[2]);
          else if (mode == FM_SIMPLE) { const double w = wa * m.ktrans; wA = mk(w, w, w); }
          else wA = mk(wa * m.permclr[0], wa * m.permclr[1], wa * m.permclr[2]);
          acc = mk(0 + (wA.x * c.x), 0 + (wA.y * c.y), 0 + (wA.z * c.z));
          if (P.hasB) {  // second child (Fresnel reflection)
            P.phase = 2;
            P.acc = acc;
            in.o = P.org; in.d = P.dB;
            if (FRAME_SLIM) { in.gen = sp; in.node = pn * 2 + 1; }  // a frame's stack index is its node's generation
            else { in.gen = P.gen + 1; in.node = P.node * 2 + 1; }
            in.ktm = (mode == FM_SIMPLE) ? -1 : P.mat;
            if (STASH_SHADE) { stash3(SL_RAYO, in.o); stash3(SL_RAYD, in.d); }
            if (CNT) ct.c[C_REFL]++;
            spawned = true;
            break;
          }
        } else {
          V wB;
          if (mode == FM_SIMPLE) { const double w = P.wb * m.krefl; wB = mk(w, w, w); }
          else wB = mk(P.wb * m.permclr[0], P.wb * m.permclr[1], P.wb * m.permclr[2]);
          const V a0 = (ph == 2) ? P.acc : mk(0, 0, 0);
          acc = mk(a0.x + (wB.x * c.x), a0.y + (wB.y * c.y), a0.z + (wB.z * c.z));
        }
        c = clampc(add(P.local, acc));
        sp--;
      }
    }
    if (!spawned) {
      if constexpr (RES_LDS<F>) {  // the finished colour waits in the lane's LDS slots (below)
        stash3(SL_RES, c);
        break;
      }
      return c;
    }
  }
  if constexpr (RES_LDS<F>) {
    lds_barrier();
    return unstash3(SL_RES);
  }
  __builtin_unreachable();
}

// ---------------------------------------------------------------------------
// Compacted shadow rays (packet kernels). calcShadowColor (myObjShader.java:98-153) traces one
// shadow ray per light for the hit being shaded. Lane by lane (trace_sample / light_sum), a
// light's shadow rays are traced by the lanes that hit something in this step of their own
// shading tree and whose spot cone holds the point (ltMult != 0): in C4 an any-hit step ran
// with 32 % of its lanes. Here the whole wave runs every shading step together
// (trace_sample_w), and the (lane, light) pairs with a shadow ray are numbered by ballot +
// prefix count -- light-major, lanes in order -- so that lane e of the wave traces pair e, up
// to 64 pairs per pass. Each pair's outcome (blocked, or how many in-place re-normalisations
// its direction went through, myRay.java:93) goes back to the shading lane by ds_bpermute, and
// that lane adds the light's terms in light order from the same operands as light_sum: the
// image is bit-identical to the lane-by-lane loop (and so are the instrumented counters).
// Selected per render by RT_RENDER_SHCOMPACT (render_kernel<..., SHC = true>): measured on
// MI355X it is bit-identical but slower on C3 / C4 / C5 (DESIGN.md §4 "Compacted shadow rays"),
// so it is not the default.
DEVI lds_u64* grpM() { return (lds_u64*)(pkB() + LDS_BYTES + SUM_BYTES); }
DEVI uint64_t lanes_below() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}
// position of the r-th (0-based) set bit of m, r < popcount(m)
DEVI int nth_bit(uint64_t m, int r) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll(m & ((1ull << w) - 1));
    if (r >= c) { r -= c; m >>= w; pos += w; }
  }
  return pos;
}
// the RNG key of a shading lane, for the lane tracing its shadow ray (pixel < 2^32, sample <
// 2^20, node < 2^12: checked by the host)
DEVI double key_pack(const Key& k) {
  return __builtin_bit_cast(double, (uint64_t)(uint32_t)k.pixel | ((uint64_t)(k.sample & 0xFFFFFu) << 32) |
                                        ((uint64_t)(k.node & 0xFFFu) << 52));
}
DEVI Key key_unpack(double v, uint64_t seed, uint32_t tsite) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  Key k;
  k.seed = seed; k.pixel = (uint32_t)b; k.sample = (uint32_t)(b >> 32) & 0xFFFFFu; k.node = (uint32_t)(b >> 52);
  k.tsite = tsite;
  return k;
}
// the shadow ray of light li from the hit point fwd, as light_sum sets it up
// (calcShadowColor :98-121): direction, distance to the light, spot fall-off.
// U: li is wave-uniform (the light record as scalar loads)
struct ShRay {
  V d;
  double dist, ltm;
};
template <uint32_t F, bool U>
DEVI ShRay shadow_ray(const SceneD& S, int li, V fwd, const Key& k) {
  const LightD& L = S.light[li];
  auto ld = [&](const double* p) { return U ? sload(p) : *p; };
  const int32_t ltype = U ? sload(&L.type) : L.type;
  double lg[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) lg[q] = ld(L.g + q);
  const V lorg = mk(ld(L.origin), ld(L.origin + 1), ld(L.origin + 2));
  const bool disk = (F & FT_LIGHTX) && ltype == 2;
  const V lo = disk ? disk_pos<U>(L, k, 0) : lorg;
  V ln = xpt(lg, lo);
  ln = nrmz(mk(ln.x - fwd.x, ln.y - fwd.y, ln.z - fwd.z));
  ShRay r;
  r.d = nrmz(ln);  // myRay ctor normalises again
  const V lo2 = disk ? disk_pos<U>(L, k, 2) : lorg;
  r.dist = sqrt((((fwd.x - lo2.x) * (fwd.x - lo2.x)) + ((fwd.y - lo2.y) * (fwd.y - lo2.y))) +
                ((fwd.z - lo2.z) * (fwd.z - lo2.z)));
  r.ltm = 1;
  if ((F & FT_LIGHTX) && ltype == 1) {  // mySpotLight.calcT_Mult (myLight.java:77-82,159-163)
    const double angle = jf::acos(-1 * dot(r.d, pld3<U>(L.orient)));
    const double inR = pld<U>(&L.innerRad), outR = pld<U>(&L.outerRad);
    r.ltm = (angle < inR) ? 1 : (angle > outR) ? 0 : (outR - angle) / pld<U>(&L.radDiff);
  }
  return r;
}
// calcShadowColor for the hits of one wave step. Every lane of the wave calls it; `hit`: this
// lane shades a hit whose point, key, normal, view direction and texture colour are in the
// stash slots (shade_pre). Returns the lane's light sum (light_sum's value).
template <bool CNT, uint32_t F>
DEVI V light_sum_w(const SceneD& S, bool hit, int32_t mat, const Key& k, Counters& ct) {
  if (!__ballot(hit)) return mk(0, 0, 0);
  const int lane = __lane_id();
  double r = 0, g = 0, b = 0;
  lds_u64* gm = grpM();
  int li0 = 0, ns = 0, n = 0;  // the pending group: lights li0 .. li0 + ns - 1 with n shadow rays
  const int nl = S.nlight;
  for (int li = 0; li <= nl; ++li) {
    uint64_t mask = 0;
    if (li < nl) {  // pass 1: which lanes have a shadow ray for light li
      double ltm = 0;
      if (hit) {
        if (CNT) ct.c[C_LIGHT]++;
        ltm = shadow_ray<F, true>(S, li, unstash3(SL_FWD), k).ltm;
        if (CNT && ltm != 0) ct.c[C_SHADOW]++;
      }
      WCNT(C_WLIGHT, 1);  // the light record: scalar loads, once per wave
      mask = __ballot(hit && ltm != 0);
    }
    const int c = __popcll(mask);
    if (li == nl || n + c > 64 || ns == GRP_MAX) {
      if (n > 0) {
        lds_barrier();
        // pass 2: lane e traces the group's e-th shadow ray (source lane, light) -> res
        int es = 0, er = 0, base = 0;
        for (int s = 0; s < ns; ++s) {
          const int cs = __popcll(uni64(gm[s]));
          if (lane >= base && lane < base + cs) { es = s; er = lane - base; }
          base += cs;
        }
        int res = -1;  // -1: blocked (or no ray); else the re-normalisations of its direction
        if (lane < n) {
          const int src = nth_bit(gm[es], er);
          const V o = mk(pkT()[SL_FWD * 64 + src], pkT()[(SL_FWD + 1) * 64 + src], pkT()[(SL_FWD + 2) * 64 + src]);
          const Key sk = key_unpack(pkT()[SL_KEY * 64 + src], k.seed, SITE_SHADOW_TIME + li0 + es);
          const ShRay sh = shadow_ray<F, false>(S, li0 + es, o, sk);
          WRay sr;
          sr.o = o; sr.d = sh.d; sr.d0 = sh.d; sr.stable = false; sr.moved = false; sr.ver = 0;
          PKSTAT(P_SH_STEP, __ballot(1));
          PROF_T0(t_shd);
#ifdef RT_PROF_NOSHADOW  // profiling builds only (tools/variant_sweep.py): results differ
          if (true) {
#else
          if (!shadowed<CNT, F, PACKET>(S, sr, sk, sh.dist, ct)) {
#endif
            renorm(sr);  // shadowRay.direction._normalize()
            res = (int)sr.ver;
          }
          PROF_ADD(t_shd, R_SHADOW);
        }
        lds_barrier();
        // pass 3: each shading lane adds its lights' terms, in light order (light_sum)
        const uint64_t below = lanes_below();
        base = 0;
        for (int s = 0; s < ns; ++s) {
          const uint64_t m = uni64(gm[s]);
          const int rs = __builtin_amdgcn_ds_bpermute((base + (int)__popcll(m & below)) << 2, res);
          base += __popcll(m);
          if (in_mask(m) && rs >= 0) {
            const int lj = li0 + s;
            const ShRay sh = shadow_ray<F, true>(S, lj, unstash3(SL_FWD), k);
            V d = sh.d;  // the direction after the scan's re-normalisations: nrmz^rs(d0)
            for (int q = 0; q < rs; ++q) d = nrmz(d);
            const LightD& L = S.light[lj];
            const V lcol = mk(sload(L.color), sload(L.color + 1), sload(L.color + 2));
            const V hn = unstash3(SL_NRM);
            const double ldp = dot(d, hn) * sh.ltm;
            if (ldp > EPS) {
              const V tx = unstash3(SL_TEX);
              r += tx.x * lcol.x * ldp;
              g += tx.y * lcol.y * ldp;
              b += tx.z * lcol.z * ldp;
            }
#ifndef RT_PROF_NOPHONG  // profiling builds only: results differ
            const MatD& mt = S.mat[mat];
            if (mt.phong != 0) {  // the specular term at shading precision (light_sum)
              const V hdw = unstash3(SL_DW);
              const V hv = mk(d.x - hdw.x, d.y - hdw.y, d.z - hdw.z);
              const double hm = mag(hv), hr = hm == 0 ? 1.0 : 1.0 / hm;
              const double hdp = (hv.x * hr * hn.x + hv.y * hr * hn.y + hv.z * hr * hn.z) * sh.ltm;
              if (hdp > EPS) {
                const double ph = pow_shade(hdp * hdp, mt.phong);
                r += mt.specular[0] * lcol.x * ph;
                g += mt.specular[1] * lcol.y * ph;
                b += mt.specular[2] * lcol.z * ph;
              }
            }
#endif
          }
        }
        lds_barrier();
      }
      li0 = li; ns = 0; n = 0;
    }
    if (li < nl) {
      gm[ns] = mask;  // wave-uniform: every lane writes the same value
      ns++;
      n += c;
    }
  }
  return mk(r, g, b);
}

// getColorAtPos (myObjShader.java:409-438) around the wave's compacted shadow rays.
// shade_pre: the hit's ambient (+ photon) and texture colours; what the light terms and the
// lanes tracing its shadow rays need goes to the stash slots.
template <bool CNT, uint32_t F>
DEVI void shade_pre(const SceneD& S, const HitRec& h, const Key& k, Counters& ct) {
  const MatD& m = S.mat[h.mat];
  double r = m.ambient[0], g = m.ambient[1], b = m.ambient[2];
  if constexpr ((F & FT_PHOTON) != 0) {
    if (!m.simple && (m.krefl == 0.0) && m.usePhotonMap) {
#ifdef RT_PROF_NOGATHER  // profiling builds only: results differ
      V ir = mk(0, 0, 0);
#else
      PROF_T0(t_ph);
      V ir = irradiance<CNT>(S, h.fwd, ct);
      PROF_ADD(t_ph, R_PHOTON);
#endif
      if (m.isCausticPhtn) { r += ir.x; g += ir.y; b += ir.z; }
      else { r += m.diffuse[0] * ir.x; g += m.diffuse[1] * ir.y; b += m.diffuse[2] * ir.z; }
    }
  }
  PROF_T0(t_tex);
  const V tex = diff_color<CNT, F>(S, m, h, k, m.simple ? 1.0 : m.diffConst, ct);
  PROF_ADD(t_tex, R_TEX);
  stash3(SL_BASE, mk(r, g, b)); stash3(SL_TEX, tex); stash3(SL_NRM, h.nrm); stash3(SL_DW, h.dw);
  stash3(SL_FWD, h.fwd); stash(SL_KEY, key_pack(k));
  lds_barrier();
}
// shade_post: the node's colour (ambient + photon + light sum) and its children, as shade_node
// after light_sum; the hit's point, normal and view direction come from the stash slots
template <bool CNT, uint32_t F>
DEVI int shade_post(const SceneD& S, int32_t mat, V ls, const Child& in, FrameOf<F>& Fr, Child& a, bool& branch,
                    Counters& ct) {
  const MatD& m = S.mat[mat];
  lds_barrier();
  const V base = unstash3(SL_BASE);
  Fr.local = mk(base.x + ls.x, base.y + ls.y, base.z + ls.z);
  branch = (in.gen < S.numRays - 2) && m.hasCaustic;
#ifdef RT_PROF_NOSECONDARY  // profiling builds only: results differ
  branch = false;
#endif
  if (!branch) return 0;
  HitRec hs;
  hs.nrm = unstash3(SL_NRM);
  hs.dw = unstash3(SL_DW);
  const V fwd = unstash3(SL_FWD);
  lds_barrier();
  a.o = fwd;
  stash3(SL_RAYO, a.o);  // the child ray goes to trace_sample_w through LDS
  a.gen = in.gen + 1;
  a.node = in.node * 2;
  if constexpr ((F & FT_TRANS) != 0) {
    bool trans = !m.simple && ((m.ktrans > 0) || (m.perm > 0.0));
    bool strans = m.simple && (m.ktrans > 0);
    if (trans || strans) {  // calcTransClr :157-276 / calcSimpleTransClr :503-631
      double ik[2];
      kt_of(S, in.ktm, ik);
      const TransOut T = trans_split(m, hs, ik, strans);
      Fr.mat = mat;
      Fr.mode = strans ? FM_SIMPLE : FM_FRESNEL;
      Fr.wa = T.omtr;
      Fr.wb = T.tr;
      if (T.doA) {
        a.d = T.refr;
        stash3(SL_RAYD, a.d);
        a.ktm = mat;
        if (CNT) ct.c[C_REFR]++;
        Fr.phase = 1;
        Fr.hasB = T.doB;
        if (T.doB) {
          Fr.dB = T.refl;
          Fr.org = fwd;
          Fr.node = in.node;
          Fr.gen = in.gen;
        }
        return T.doB ? 2 : 1;
      }
      if (T.doB) {  // only the reflection child: spawn it as "B"
        a.d = T.refl;
        stash3(SL_RAYD, a.d);
        a.node = in.node * 2 + 1;
        a.ktm = strans ? -1 : mat;
        if (CNT) ct.c[C_REFL]++;
        Fr.phase = 3;
        return 1;
      }
      return 0;
    }
  }
  if (m.krefl > 0.0) {  // calcReflClr :278-294
    V back = mk(hs.dw.x * -1, hs.dw.y * -1, hs.dw.z * -1);
    V rd = refl_dir(back, hs.nrm);
    if (dot(rd, hs.nrm) >= 0) {
      a.d = rd;
      stash3(SL_RAYD, a.d);
      a.ktm = -1;
      Fr.phase = 1;
      Fr.mat = mat;
      if constexpr ((F & FT_TRANS) != 0) {
        Fr.mode = FM_REFL;
        Fr.hasB = 0;
      }
      if (CNT) ct.c[C_REFL]++;
      return 1;
    }
  }
  return 0;
}

// trace_sample with the whole wave in step: every lane runs the loop until no lane of the wave
// has a ray left (`live`), so all 64 lanes reach light_sum_w together and can trace the step's
// shadow rays. Same shading tree, order and arithmetic per lane as trace_sample.
template <bool CNT, uint32_t F>
DEVI V trace_sample_w(const SceneD& S, V org, V dir, Key k, bool live, Counters& ct) {
  FrameOf<F> fr[MAX_FRAMES];
  int sp = 0;
  Child in;
  in.o = org; in.d = dir; in.node = 1; in.gen = 0; in.ktm = -1;
  V out = mk(0, 0, 0);
  if (live) { stash3(SL_RAYO, in.o); stash3(SL_RAYD, in.d); }
  while (__ballot(live)) {
    bool hit = false;
    int32_t mat = 0;
    V c = mk(0, 0, 0);
    if (live) {
      lds_barrier();
      in.o = unstash3(SL_RAYO); in.d = unstash3(SL_RAYD);
      WRay w;
      w.o = in.o; w.d = nrmz(in.d); w.d0 = w.d; w.stable = false; w.moved = false; w.ver = 0;  // myRay ctor
      k.node = in.node;
      PKSTAT(P_RAY_STEP, __ballot(1));
      const Best bh = closest<CNT, F, PACKET>(S, w, k, ct);
      if (bh.t == DMAX) {
        PROF_T0(t_bg);
        c = background<CNT, F>(S, w, ct);
        PROF_ADD(t_bg, R_BG);
      } else {
        PROF_T0(t_hit);
        const HitRec h = make_hit<F>(S, bh, w, k);
        PROF_ADD(t_hit, R_HIT);
        PROF_T0(t_sh);
        shade_pre<CNT, F>(S, h, k, ct);
        PROF_ADD(t_sh, R_SHADE);
        mat = h.mat;
        hit = true;
      }
    }
    PROF_T0(t_ls);
    const V ls = light_sum_w<CNT, F>(S, hit, mat, k, ct);
    PROF_ADD(t_ls, R_LIGHT);
    if (live) {
      bool spawned = false;
      if (hit) {
        bool branch;
        Child a;
        FrameOf<F>& Fr = fr[sp];
        const int nch = shade_post<CNT, F>(S, mat, ls, in, Fr, a, branch, ct);
        if (nch > 0 && sp < MAX_FRAMES) {
          sp++;
          in = a;  // its o / d are in the LDS slots (shade_post)
          spawned = true;
        } else {
          c = branch ? clampc(add(Fr.local, mk(0, 0, 0))) : clampc(Fr.local);  // no child: acc stayed 0
        }
      }
      // deliver finished colours upward (trace_sample)
      while (!spawned && sp > 0) {
        FrameOf<F>& P = fr[sp - 1];
        if constexpr ((F & FT_TRANS) == 0) {  // the only child has returned
          const double* wA = S.mat[P.mat].kreflclr;
          V acc = mk(0 + (wA[0] * c.x), 0 + (wA[1] * c.y), 0 + (wA[2] * c.z));
          c = clampc(add(P.local, acc));
          sp--;
        } else {
          const MatD& m = S.mat[P.mat];
          const uint8_t ph = P.phase, mode = P.mode;
          V acc;
          if (ph == 1) {
            V wA;
            if (mode == FM_REFL) wA = mk(m.kreflclr[0], m.kreflclr[1], m.kreflclr[2]);
            else if (mode == FM_SIMPLE) { const double w = P.wa * m.ktrans; wA = mk(w, w, w); }
            else wA = mk(P.wa * m.permclr[0], P.wa * m.permclr[1], P.wa * m.permclr[2]);
            acc = mk(0 + (wA.x * c.x), 0 + (wA.y * c.y), 0 + (wA.z * c.z));
            if (P.hasB) {  // second child (Fresnel reflection)
              P.phase = 2;
              P.acc = acc;
              in.o = P.org; in.d = P.dB; in.gen = P.gen + 1; in.node = P.node * 2 + 1;
              in.ktm = (mode == FM_SIMPLE) ? -1 : P.mat;
              stash3(SL_RAYO, in.o); stash3(SL_RAYD, in.d);
              if (CNT) ct.c[C_REFL]++;
              spawned = true;
              break;
            }
          } else {
            V wB;
            if (mode == FM_SIMPLE) { const double w = P.wb * m.krefl; wB = mk(w, w, w); }
            else wB = mk(P.wb * m.permclr[0], P.wb * m.permclr[1], P.wb * m.permclr[2]);
            const V a0 = (ph == 2) ? P.acc : mk(0, 0, 0);
            acc = mk(a0.x + (wB.x * c.x), a0.y + (wB.y * c.y), a0.z + (wB.z * c.z));
          }
          c = clampc(add(P.local, acc));
          sp--;
        }
      }
      if (!spawned) { out = c; live = false; }
    }
  }
  return out;
}

// XCD-aware tile order. Workgroups are dealt round-robin to the 8 XCDs (block b -> XCD
// b % 8), each with its own L2. With XCD_CHUNKS = k > 0 the row-major tile list is cut
// into 8k contiguous chunks and XCD x renders chunks x, x+8, ...: each L2 then sees a
// few image bands (and the part of the scene they show) instead of the whole frame.
#ifndef RT_XCD_CHUNKS
#define RT_XCD_CHUNKS 0
#endif
static constexpr int XCD_CHUNKS = RT_XCD_CHUNKS;
__host__ __device__ inline int xcd_grid(int ntiles) {
  if constexpr (XCD_CHUNKS == 0) return ntiles;
  const int nch = 8 * (XCD_CHUNKS ? XCD_CHUNKS : 1), csz = (ntiles + nch - 1) / nch;
  return nch * csz;
}
DEVI int tile_of_block(int b, int ntiles) {
  if constexpr (XCD_CHUNKS == 0) return b;
  const int nch = 8 * (XCD_CHUNKS ? XCD_CHUNKS : 1), csz = (ntiles + nch - 1) / nch;
  const int xcd = b & 7, slot = b >> 3;
  const int t = ((slot / csz) * 8 + xcd) * csz + slot % csz;
  return t < ntiles ? t : -1;
}

#ifndef RT_RENDER_WAVES
#define RT_RENDER_WAVES 4
#endif
// where a lane's pixel is: sample lane j of pixel pl of the wave's tile
struct PixGeo {
  int j, pl, ci, col, ri, row;
  bool valid;
};
template <uint32_t F>
DEVI PixGeo pix_geo(int lane, int tile, int tilesX, int ncols, const ParamsD& P) {
  PixGeo g;
  g.j = lane & (P.G - 1);
  g.pl = lane / P.G;
  const int tx = tile % tilesX, ty = tile / tilesX;
  g.ci = tx * P.tw + g.pl % P.tw;  // column index within this render's columns
  g.col = (F & FT_PASS) ? g.ci * P.colStep : g.ci;
  g.ri = ty * P.th + g.pl / P.tw;  // row index within this render's rows
  g.valid = g.ci < ncols && g.ri < P.nrows;
  const int band = uni_here(P.band);  // (the division's reciprocal is not kept across the sample loop)
  g.row = band == 1 ? P.row0 + g.ri * P.rowStep : P.row0 + (g.ri / band) * P.rowStep * band + g.ri % band;
  return g;
}
// the lane index as an opaque value: what is derived from it is recomputed where it is used
// instead of being hoisted out of the sample loop and kept (spilled) across the shading tree
DEVI int opaque_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}
#ifdef RT_PROF_TIMELINE  // profiling builds only (tools/timeline.py): per-workgroup start/end clock + HW ids
__device__ unsigned long long* rt_tl_buf;
#endif
// C3's and C5's render variants are instantiated in render_minreg.hip, compiled with the
// register-minimising machine scheduler (C3 -1.2 %, C5 -1 %; C4's variant loses 6 % with it, so
// it and the others stay in trace.hip). Profiling builds keep every variant in trace.hip (their
// counters are module globals read through trace.hip's module).
#if defined(RT_PROF_PKSTAT) || defined(RT_PROF_REGIONS) || defined(RT_PROF_TIMELINE) || defined(RT_NO_SPLIT_TU)
#define RT_SPLIT_TU 0
#else
#define RT_SPLIT_TU 1
#endif
static constexpr uint32_t F_C5 = FT_PRIM | FT_TRANS | FT_PHOTON | FT_LIGHTX;
// SHC: the shading steps of a wave run in step and their shadow rays are traced compacted
// (trace_sample_w / light_sum_w) instead of lane by lane (trace_sample)
template <bool CNT, uint32_t F, bool SHC = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_RENDER_WAVES)))
render_kernel(SceneD S, ParamsD P, float* __restrict__ rgb, int32_t* __restrict__ argb, unsigned long long* __restrict__ gcount) {
  constexpr bool SH_COMPACT = SHC && STASH_SHADE;
  // One wave = a tw x th pixel tile x G sample lanes per pixel. Samples of one pixel are
  // nearly the same ray, so the G lanes of a pixel traverse the same nodes (coherent
  // loads, little divergence). Lane j of a pixel traces samples j, j+G, ...; each round's
  // G colours go through LDS and the pixel's first lane adds them in sample order, so
  // the per-pixel sum is the reference's sequential sum (myScene.java:1451-1460).
  double* cbuf = rt_lds;  // 64 x 4 doubles (colour, traced), aliases the traversal stack
  const int lane = threadIdx.x;
  const int G = P.G;
  // columns 0, colStep, ... of a refine pass; the other kernels render every column (the
  // column-step arithmetic alone cost the C3 kernel 2.4 %)
  const int ncols = (F & FT_PASS) ? (P.W + P.colStep - 1) / P.colStep : P.W;
  const int tilesX = (ncols + P.tw - 1) / P.tw;
  int tile = tile_of_block(blockIdx.x, tilesX * ((P.nrows + P.th - 1) / P.th));
  if (tile < 0) return;  // padding block of the XCD mapping (whole workgroup)
  if (P.order) tile = P.order[tile];
  const unsigned long long tl0 = __builtin_amdgcn_s_memrealtime();  // wave start (tcost / timeline)
  PROF_T0(tk0);
#ifdef RT_PROF_REGIONS
  if (lane < R_N) profL()[lane] = 0;
#endif
  Counters ct;
  if (CNT)
    for (int i = 0; i < P_N; ++i) ct.c[i] = 0;
  Key k;
  k.seed = P.seed;
  k.tsite = SITE_TIME;
  const int n = P.spp;
  const bool dof = (F & FT_DOF) && S.dof && !((F & FT_CAMX) && P.cam != 0);
  V fpt = mk(0, 0, 0), lc = mk(0, 0, 0);
  if (dof && pix_geo<F>(lane, tile, tilesX, ncols, P).valid) {  // shootMultiDpthOfFldRays (myScene.java:1386-1406)
    const PixGeo g = pix_geo<F>(lane, tile, tilesX, ncols, P);
    const double rayY = (-1 * (g.row - P.H / 2.0)), rayX = g.col - P.W / 2.0;
    lc = nrmz(mk(rayX, rayY, P.viewZ));
    // ray(eye, lc) hits the focal plane z = -focal (myPlane, identity CTM): the ctor and
    // getTransformedRay both normalise, then (o,1),(d,0) go through the identity inverse
    const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    V ld = nrmz(nrmz(lc));
    V fo = xpt(I, mk(0, 0, 0)), fd = xvec(I, ld);
    V fN = mk(0, 0, 1);
    double pr = dot(fN, fd);
    double t = -(dot(fN, fo) + S.lensFocal) / pr;
    fpt = mk(fd.x * t + fo.x, fd.y * t + fo.y, fd.z * t + fo.z);
  }
  // per-pixel sums. SUMS_LDS variants keep them in LDS across the shading trees -- G >= 2 in
  // sums[] (sample order), G == 1 (spp = 1, one round) as the lane's colour in cbuf; the others
  // in registers (rs / gs / bs; the 1-spp non-DOF path keeps its one colour there). Which is
  // faster depends on the variant's register allocation (measured: C3's F = 0 gains, C4's
  // transparent variant loses 6 %).
  constexpr bool SUMS_LDS = (F & FT_TRANS) == 0 || (RT_SUMS_LDS_TRANS != 0 && (F & FT_PHOTON) == 0);
  double rs = 0, gs = 0, bs = 0;
  lds_f64* sums = (lds_f64*)((lds_u8*)rt_lds + LDS_BYTES);
  if (SUMS_LDS && G > 1 && (lane & (G - 1)) == 0) {
    const int p = lane / G;
    sums[3 * p] = 0; sums[3 * p + 1] = 0; sums[3 * p + 2] = 0;
  }
  for (int s0 = 0; s0 < n; s0 += G) {
    const PixGeo g = pix_geo<F>(opaque_lane(lane), tile, tilesX, ncols, P);
    const int j = g.j, pl = g.pl, col = g.col, row = g.row;
    const bool valid = g.valid;
    const double rayY = (-1 * (row - uni_here(P.H) / 2.0));
    const double rayX = col - uni_here(P.W) / 2.0;
    k.pixel = (uint64_t)row * (uint64_t)P.W + (uint64_t)col;
    const int s = s0 + j;
    V cc = mk(0, 0, 0);
    bool traced = false;  // a fisheye sample outside the image circle adds nothing (myScene.java:1571)
    V o = mk(0, 0, 0), d = mk(0, 0, 0);
    if (valid && s < n) {
      traced = true;
      if ((F & FT_CAMX) && P.cam == 1) {  // myFishEyeScene: draw (1 spp) :1605-1622 / shootMultiRays :1562-1583
        double xVal, yVal, rSq;
        if (n == 1) {
          yVal = (row + P.yStart) * P.fishMult;
          const double ySq = yVal * yVal;
          xVal = (col + P.xStart) * P.fishMult;
          rSq = xVal * xVal + ySq;
          traced = !(rSq > 1);  // outside: blkColor
        } else {
          yVal = ((row + P.yStart) + rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5)) * P.fishMult;
          xVal = ((col + P.xStart) + rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5)) * P.fishMult;
          rSq = yVal * yVal + xVal * xVal;
          traced = rSq <= 1;
        }
        const double r = sqrt(rSq), theta = r * P.aperHalf, phi = atan2(-yVal, xVal), sTh = jf::sin(theta);
        o = mk(0, 0, 0);
        d = mk(sTh * jf::cos(phi), sTh * jf::sin(phi), -jf::cos(theta));
      } else if ((F & FT_CAMX) && P.cam == 2) {  // myOrthoScene: draw :1704-1745 / shootMultiRays :1690-1702
        const double rayYOffset = P.H / 2.0, rayXOffset = P.W / 2.0;
        double rx, ry;
        if (n == 1) {
          ry = P.orthPerRow * (-1 * (row - rayYOffset));
          rx = P.orthPerCol * (col - rayXOffset);
        } else {
          const double yB = P.orthPerRow * ((-1 * (row - rayYOffset)) - .5), xB = P.orthPerCol * (col - rayXOffset - .5);
          ry = yB + (P.orthPerRow * rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5));
          rx = xB + (P.orthPerCol * rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5));
        }
        o = mk(rx, ry, 0);
        d = mk(0, 0, -1);
      } else if (dof) {
        double th = rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_DOF_ANG, 0, 0, TWO_PI_F);
        V tt = nrmz(rot_axis(mk(0, 1, 0), mk(0, 0, -1), th));
        double mm = rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_DOF_RAD, 0, 0, S.lensRadius);
        tt = mk(tt.x * mm, tt.y * mm, tt.z * mm);
        o = mk(tt.x + lc.x, tt.y + lc.y, tt.z + lc.z);
        d = sub(fpt, o);
      } else if (n == 1) {  // myFOVScene.draw 1-spp path (:1498-1508): no jitter, no averaging
        o = mk(0, 0, 0);
        d = mk(rayX, rayY, P.viewZ);
      } else {  // shootMultiRays (:1447-1462): y jitter drawn before x
        double ry = rayY + rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5);
        double rx = rayX + rng(P.seed, k.pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5);
        o = mk(0, 0, 0);
        d = mk(rx, ry, uni_here(P.viewZ));
      }
      if (!SH_COMPACT && traced) {
        Key ks = k;
        ks.sample = (uint32_t)s;
        if (CNT) ct.c[C_CAMERA]++;
        PROF_T0(t_smp);
#ifdef RT_PROF_NOSAMPLE  // profiling builds only (tools/variant_sweep.py): the camera setup, sums and output alone
        cc = mk(d.x * 1e-3, d.y * 1e-3, 0);
#else
        cc = trace_sample<CNT, F>(S, o, d, ks, ct);
#endif
        PROF_ADD(t_smp, R_SAMPLE);
      }
    }
    if constexpr (SH_COMPACT) {  // every lane of the wave: the shading steps run in step
      Key ks = k;
      ks.sample = (uint32_t)s;
      if (CNT && traced) ct.c[C_CAMERA]++;
      PROF_T0(t_smp);
      cc = trace_sample_w<CNT, F>(S, o, d, ks, traced, ct);
      PROF_ADD(t_smp, R_SAMPLE);
    }
    if (G == 1) {  // one sample per pixel (G = 1 only for spp = 1): one round
      if constexpr (SUMS_LDS) {  // its colour waits in cbuf
        cbuf[4 * lane + 0] = cc.x;
        cbuf[4 * lane + 1] = cc.y;
        cbuf[4 * lane + 2] = cc.z;
        cbuf[4 * lane + 3] = traced ? 1.0 : 0.0;
      } else {
        if (n == 1 && !dof) { rs = cc.x; gs = cc.y; bs = cc.z; }
        else if (traced) { rs += cc.x; gs += cc.y; bs += cc.z; }
      }
    } else {
      cbuf[4 * lane + 0] = cc.x;
      cbuf[4 * lane + 1] = cc.y;
      cbuf[4 * lane + 2] = cc.z;
      cbuf[4 * lane + 3] = traced ? 1.0 : 0.0;
      __syncthreads();
      if (j == 0) {
        const int m = (n - s0) < G ? (n - s0) : G;
        double sr = rs, sg = gs, sb = bs;
        if (SUMS_LDS) { sr = sums[3 * pl]; sg = sums[3 * pl + 1]; sb = sums[3 * pl + 2]; }
        for (int q = 0; q < m; ++q) {
          const double* b = cbuf + 4 * (pl * G + q);
          if (b[3] != 0) { sr += b[0]; sg += b[1]; sb += b[2]; }
        }
        if (SUMS_LDS) { sums[3 * pl] = sr; sums[3 * pl + 1] = sg; sums[3 * pl + 2] = sb; }
        else { rs = sr; gs = sg; bs = sb; }
      }
      __syncthreads();
    }
  }
  const PixGeo g = pix_geo<F>(opaque_lane(lane), tile, tilesX, ncols, P);
  if (SUMS_LDS && G > 1 && g.j == 0) { rs = sums[3 * g.pl]; gs = sums[3 * g.pl + 1]; bs = sums[3 * g.pl + 2]; }
  if (SUMS_LDS && G == 1) {
    const double* b = cbuf + 4 * lane;
    if (n == 1 && !dof) { rs = b[0]; gs = b[1]; bs = b[2]; }  // the colour as traced (no averaging)
    else if (b[3] != 0) { rs = 0 + b[0]; gs = 0 + b[1]; bs = 0 + b[2]; }  // the sum of one sample
  }
  if (g.valid && g.j == 0) {
    V c = (n == 1 && !dof) ? mk(rs, gs, bs) : clampc(mk(rs / n, gs / n, bs / n));
    const size_t o = (size_t)g.ri * ncols + g.ci;
    if (rgb) {
      rgb[3 * o + 0] = (float)c.x;
      rgb[3 * o + 1] = (float)c.y;
      rgb[3 * o + 2] = (float)c.z;
    }
    if (argb) {  // myColor.getInt (myObjShader.java:671)
      uint32_t v = (uint32_t)(255u << 24) + ((uint32_t)jd2i(c.x * 255) << 16) + ((uint32_t)jd2i(c.y * 255) << 8) +
                   (uint32_t)jd2i(c.z * 255);
      argb[o] = (int32_t)v;
    }
  }
  if (CNT) {
    for (int i = 0; i < C_N; ++i)
      if (ct.c[i]) atomicAdd(&gcount[i], (unsigned long long)ct.c[i]);
#ifdef RT_PROF_PKSTAT
    for (int i = C_N; i < P_N; ++i)
      if (ct.c[i]) atomicAdd(&rt_pk_stat[i - C_N], (unsigned long long)ct.c[i]);
#endif
  }
  if (!CNT && P.tcost && lane == 0) P.tcost[tile] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - tl0);
#ifdef RT_PROF_REGIONS
  if (!CNT) {
    PROF_ADD(tk0, R_KERNEL);
    if (lane < R_N) atomicAdd(&rt_prof_reg[lane], (unsigned long long)profL()[lane]);
  }
#endif
#ifdef RT_PROF_TIMELINE
  if (!CNT && lane == 0 && rt_tl_buf) {
    unsigned long long* b = rt_tl_buf + 4 * (size_t)blockIdx.x;
    b[0] = tl0;
    b[1] = __builtin_amdgcn_s_memrealtime();
    b[2] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_ID
    b[3] = ((unsigned)__builtin_amdgcn_s_getreg(20 | (3 << 11))) | ((unsigned long long)tile << 8);  // XCC_ID
  }
#endif
}

#ifndef RT_MINREG_TU
// The photon gather alone (rt_photon_gather): lane i returns getIrradianceFromPhtnTree at point i
// through the render kernel's gather (counting selection, packet scans, exact-tie replay).
__global__ void __launch_bounds__(64) gather_kernel(SceneD S, const double* __restrict__ pts, double* __restrict__ out,
                                                    int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  Counters ct;
  const V ir = irradiance<false>(S, mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), ct);
  out[3 * i] = ir.x; out[3 * i + 1] = ir.y; out[3 * i + 2] = ir.z;
}
#endif

#if RT_SPLIT_TU && !defined(RT_MINREG_TU)
extern template __global__ void render_kernel<false, 0u>(SceneD, ParamsD, float*, int32_t*, unsigned long long*);
extern template __global__ void render_kernel<false, F_C5>(SceneD, ParamsD, float*, int32_t*, unsigned long long*);
#endif
#ifndef RT_MINREG_TU  // the other kernels: trace.hip only
// Tile cost probe for the dispatch schedule: one lane per tile traces the tile's first
// pixel's un-jittered camera ray (closest hit only) and reports the work it counted.
// Only the ORDER in which tiles are dispatched depends on it, never a pixel.
template <uint32_t F>
__global__ void __launch_bounds__(64) probe_kernel(SceneD S, ParamsD P, uint32_t* __restrict__ cost, int ntiles) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= ntiles) return;
  const int ncols = (P.W + P.colStep - 1) / P.colStep;
  const int tilesX = (ncols + P.tw - 1) / P.tw;
  const int col = (t % tilesX) * P.tw * P.colStep, ri = (t / tilesX) * P.th;
  const int row = P.row0 + (ri / P.band) * P.rowStep * P.band + ri % P.band;
  Counters ct;
  for (int i = 0; i < P_N; ++i) ct.c[i] = 0;
  WRay w;
  w.o = mk(0, 0, 0);
  w.d = nrmz(mk(col - P.W / 2.0, -1 * (row - P.H / 2.0), P.viewZ));
  w.d0 = w.d; w.stable = false; w.moved = false; w.ver = 0;
  Key k;
  k.seed = P.seed; k.pixel = (uint64_t)row * P.W + col; k.sample = 0; k.node = 1; k.tsite = SITE_TIME;
  closest<true, F>(S, w, k, ct);
  cost[t] = (uint32_t)(1 + ct.c[C_NODE] + ct.c[C_TRI] + ct.c[C_QUAD] + ct.c[C_IMPLICIT] + ct.c[C_TOP]);
}

// ---------------------------------------------------------------------------
// photon pre-pass (myScene.sendCausticPhotons :952-998 / sendDiffusePhotons :1000-1091):
// one lane per emitted photon (light-major, photon index minor). Each lane writes
// its stored photons into PH_SLOTS slots in path order; the host compacts them in
// (light, index, slot) order -- the reference's photon_list insertion order.
static constexpr int PH_SLOTS = 6;
static constexpr int PH_MAXTRY = 4096;  // rejection-sampling cap (reached with probability ~0)
struct PhotonOut {
  double pos[3];
  double pwr[3];
};
// genRndPhtnRay (myLight.java:104-107 point, :165-185 spot, :229-242 disk; getRandDir :59-74)
DEVI void photon_ray(const LightD& L, uint64_t seed, uint64_t i, V& o, V& d) {
  uint32_t k = 0, li = (uint32_t)L.index;
  if (L.type == 0) {
    double x, y, z, sq;
    int tries = 0;
    do {
      x = rng(seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      y = rng(seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      z = rng(seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      sq = (x * x) + (y * y) + (z * z);
    } while (((sq > 1.0) || (sq < EPS)) && ++tries < PH_MAXTRY);
    double m = sqrt(sq);
    d = mk(x / m, y / m, z / m);
    o = xpt(L.g, ld3(L.origin));
    return;
  }
  if (L.type == 1) {
    double checkProb = rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, 1), angle, prob;
    int tries = 0;
    do {
      angle = rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, L.outerRad);
      prob = (angle < L.innerRad) ? 1 : (angle > L.outerRad) ? 0 : (L.outerRad - angle) / L.radDiff;
    } while (prob > checkProb && ++tries < PH_MAXTRY);
    V t = nrmz(rot_axis(ld3(L.orient), ld3(L.tangent), angle));
    d = rot_axis(t, ld3(L.orient), rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, TWO_PI_F));
    o = xpt(L.g, ld3(L.origin));
    return;
  }
  double angle, prob;
  int tries = 0;
  do {
    angle = rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, PI_D);
    prob = (angle < 0) ? 1 : (angle > PI_D) ? 0 : (PI_D - angle) / PI_D;
  } while (prob > rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, 1) && ++tries < PH_MAXTRY);
  V dd = nrmz(rot_axis(ld3(L.orient), ld3(L.tangent), angle));
  d = rot_axis(dd, ld3(L.orient), rng(seed, i, li, 0, SITE_PH_DIR, k++, 0, TWO_PI_F));
  Key kk;
  kk.seed = seed; kk.pixel = i; kk.sample = li; kk.node = 0; kk.tsite = SITE_PH_TIME;
  o = xpt(L.g, disk_pos(L, kk, 0));
}
// findCausticRayHit (myObjShader.java:461-478) with calcTransRay / calcReflRay
DEVI bool caustic_ray(const SceneD& S, const HitRec& h, int32_t inKtm, int gen, double pwr[3], Child& out) {
  const MatD& m = S.mat[h.mat];
  if (!((gen < 4) && m.hasCaustic)) return false;  // numPhotonRays = 4
  double pmul[3] = {1.0, 1.0, 1.0};
  bool ok = false;
  if ((m.ktrans > 0.0) || (m.perm > 0.0)) {
    pmul[0] = m.phtnPermClr[0]; pmul[1] = m.phtnPermClr[1]; pmul[2] = m.phtnPermClr[2];
    double ik[2];
    kt_of(S, inKtm, ik);
    TransOut T = trans_split(m, h, ik, false);
    out.d = (T.omtr > EPS) ? T.refr : T.refl;
    out.ktm = h.mat;
    ok = true;
  } else if (m.krefl > 0.0) {
    pmul[0] = pmul[1] = pmul[2] = m.krefl;
    out.d = refl_dir(mk(h.dw.x * -1, h.dw.y * -1, h.dw.z * -1), h.nrm);
    out.ktm = -1;
    ok = true;
  }
  for (int c = 0; c < 3; ++c) pwr[c] = pwr[c] * pmul[c];
  out.o = h.fwd;
  out.gen = gen + 1;
  return ok;
}
DEVI void new_wray(WRay& w, V o, V d) {
  w.o = o; w.d = nrmz(d); w.d0 = w.d; w.stable = false; w.moved = false; w.ver = 0;
}

// Lane gid of a launch covers photon (light li, index i) of the shard [first, first+count)
// of every light, light-major: g = gBase + gid, li = g / count, i = first + g % count.
// F: FT_ALL, or FT_ALL without FT_INST for scenes without instances
template <uint32_t F>
__global__ void __launch_bounds__(64) photon_kernel(SceneD S, uint64_t seed, long first, long count, long gBase,
                                                   long nLanes, int caustic, double pwrMult,
                                                   PhotonOut* __restrict__ out, int* __restrict__ cnt) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nLanes) return;
  const long g = gBase + gid;
  const int li = (int)(g / count);
  const uint64_t i = (uint64_t)(first + g % count);
  const LightD& L = S.light[li];
  Counters ct;
  int n = 0;
  PhotonOut* slot = out + gid * PH_SLOTS;
  double pwr[3] = {L.color[0] * pwrMult, L.color[1] * pwrMult, L.color[2] * pwrMult};
  Key k;
  k.seed = seed; k.pixel = i; k.sample = (uint32_t)li; k.node = 0; k.tsite = SITE_PH_TIME;
  WRay w;
  V po, pd;
  photon_ray(L, seed, i, po, pd);
  new_wray(w, po, pd);
  int32_t kt = -1;  // the ray's medium (Child.ktm)
  int gen = 0;
  Best b = closest<false, F>(S, w, k, ct);
  if (b.t == DMAX) { cnt[gid] = 0; return; }
  HitRec h = make_hit<F>(S, b, w, k);
  if (caustic) {
    if (!S.mat[h.mat].hasCaustic) { cnt[gid] = 0; return; }
    int rgen = 0;
    bool hit = true;
    do {
      Child c;
      double cur[3] = {pwr[0], pwr[1], pwr[2]};
      if (caustic_ray(S, h, kt, gen, cur, c)) {
        for (int q = 0; q < 3; ++q) pwr[q] = cur[q];
        kt = c.ktm;
        rgen = c.gen;
        k.node = (uint32_t)rgen;
        new_wray(w, c.o, c.d);
        b = closest<false, F>(S, w, k, ct);
        hit = b.t != DMAX;
        if (hit) { h = make_hit<F>(S, b, w, k); gen = rgen; }
      } else {
        hit = false;
      }
    } while (hit && S.mat[h.mat].hasCaustic && rgen <= 4);
    if (hit && rgen <= 4) {
      for (int q = 0; q < 3; ++q) { slot[0].pos[q] = (&h.fwd.x)[q]; slot[0].pwr[q] = pwr[q]; }
      n = 1;
    }
    cnt[gid] = n;
    return;
  }
  bool done = false, firstDiff = true, hit = true;
  uint32_t bounce = 0;
  do {
    bounce++;
    const MatD& m = S.mat[h.mat];
    if (m.krefl == 0) {
      double prob = 0;
      uint32_t kk = 0;
      if (!firstDiff) {
        if (n < PH_SLOTS) {
          for (int q = 0; q < 3; ++q) { slot[n].pos[q] = (&h.fwd.x)[q]; slot[n].pwr[q] = pwr[q]; }
          n++;
        }
        prob = rng(seed, i, (uint32_t)li, bounce, SITE_PH_BOUNCE, kk++, 0, 1.0);
      }
      firstDiff = false;
      if (prob < m.avgDiffClr) {
        double x = 0, y = 0, sq;
        int tries = 0;
        do {
          x = rng(seed, i, (uint32_t)li, bounce, SITE_PH_BOUNCE, kk++, -1.0, 1.0);
          y = rng(seed, i, (uint32_t)li, bounce, SITE_PH_BOUNCE, kk++, -1.0, 1.0);
          sq = (x * x) + (y * y);
        } while (((sq >= 1.0) || (sq < EPS)) && ++tries < PH_MAXTRY);
        double z = sqrt(1 - (sq));
        V nn = h.nrm;
        double nx = nn.x * nn.x, ny = nn.y * nn.y, nz = nn.z * nn.z;
        V tv = ((nx > ny) && (nx > nz)) ? mk(0, 0, 1) : mk(1, 0, 0);
        V p_ = cross(nn, tv), q_ = cross(p_, nn);
        nn = mk(nn.x * z, nn.y * z, nn.z * z);
        p_ = mk(p_.x * x, p_.y * x, p_.z * x);
        q_ = mk(q_.x * y, q_.y * y, q_.z * y);
        V bd = nrmz(mk(nn.x + p_.x + q_.x, nn.y + p_.y + q_.y, nn.z + p_.z + q_.z));
        for (int q = 0; q < 3; ++q) pwr[q] = pwr[q] * m.phtnDiffScl[q];
        gen = gen + 1;
        k.node = bounce;
        new_wray(w, h.fwd, bd);
        kt = -1;
        b = closest<false, F>(S, w, k, ct);
        hit = b.t != DMAX;
        if (hit) h = make_hit<F>(S, b, w, k);
      } else {
        done = true;
      }
    } else {
      Child c;
      double cur[3] = {pwr[0], pwr[1], pwr[2]};
      if (caustic_ray(S, h, kt, gen, cur, c)) {
        for (int q = 0; q < 3; ++q) pwr[q] = cur[q];
        kt = c.ktm;
        gen = c.gen;
        k.node = bounce;
        new_wray(w, c.o, c.d);
        b = closest<false, F>(S, w, k, ct);
        hit = b.t != DMAX;
        if (hit) h = make_hit<F>(S, b, w, k);
      } else {
        hit = false;
      }
    }
  } while (hit && !done && gen <= 4);
  cnt[gid] = n;
}

#endif  // RT_MINREG_TU
}  // namespace dv
}  // namespace rt
