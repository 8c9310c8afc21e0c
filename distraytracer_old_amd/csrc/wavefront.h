// Level-synchronous shading (RT_RENDER_WAVEFRONT, DESIGN.md §4 "Level-synchronous shading").
//
// reflectRay (myScene.java:907-914) evaluates a camera sample's shading tree depth first: each hit's
// getColorAtPos (myObjShader.java:409-438) spawns up to two children (calcReflClr :278-294,
// calcTransClr :157-276) and folds their colours into its own, clamping per level (Q8). The
// monolithic render kernel restates that as a per-lane post-order loop with a frame stack
// (trace_sample). Here the tree is cut into LEVELS: one launch traces and shades every ray of one
// generation of the tree for a chunk of samples, all lanes of a wave holding rays of that level --
// the children a wave spawns are compacted into the next level's queue by ballot + mbcnt prefix
// counts (one atomic add per wave) -- and each hit that has children leaves its frame (the
// node's local colour, the Fresnel split's two scalars, material, parent link) in a per-level
// record array in HBM. When no rays are left, fold launches walk the levels bottom up: a node's
// colour is the reference's clamp(local + weighted children) formed exactly as trace_sample forms
// it, written into its parent's child slot; level 0 leaves one colour per sample, and a last
// launch sums every pixel's samples in sample order (myScene.java:1451-1460). The RNG is keyed
// (pixel, sample, tree node), so the order rays are traced in changes nothing: the image is the
// monolithic kernel's bit for bit.
#pragma once

namespace rt {
namespace dv {

struct WfRay {  // a ray waiting for its level: 80 B
  double o[3], d[3];
  uint64_t pixel;
  uint32_t sample, node;
  int32_t gen, ktm;
  int32_t parent;  // the parent's record (previous level) << 1 | side (0: child A, 1: child B)
  int32_t pad;
};
struct WfNode {  // a shaded hit with children: the frame trace_sample keeps on its stack
  double local[3];
  double wa, wb;       // Fresnel / simple split: omtr, tr
  double cA[3], cB[3]; // the children's colours, written by the children (or their folds)
  int32_t mat;
  int32_t parent;      // previous-level record << 1 | side; level 0: unused (the record is the sample's)
  uint8_t kind;        // 0: no children (nothing to fold), 1: a frame
  uint8_t phase, mode, hasB;
  int32_t pad;
};
static_assert(sizeof(WfRay) == 80 && sizeof(WfNode) == 104, "wavefront records");

#ifndef RT_WF_WAVES
#define RT_WF_WAVES 4
#endif

// camera ray of sample s of a pixel (render_kernel's camera code, myScene.java:1386-1462, 1562-1745)
template <uint32_t F>
DEVI bool wf_camera(const SceneD& S, const ParamsD& P, const PixGeo& g, int s, bool dof, V fpt, V lc, uint64_t pixel,
                    V& o, V& d) {
  const int n = P.spp;
  const int row = g.row, col = g.col;
  const double rayY = (-1 * (row - P.H / 2.0)), rayX = col - P.W / 2.0;
  bool traced = true;
  if ((F & FT_CAMX) && P.cam == 1) {
    double xVal, yVal, rSq;
    if (n == 1) {
      yVal = (row + P.yStart) * P.fishMult;
      const double ySq = yVal * yVal;
      xVal = (col + P.xStart) * P.fishMult;
      rSq = xVal * xVal + ySq;
      traced = !(rSq > 1);
    } else {
      yVal = ((row + P.yStart) + rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5)) * P.fishMult;
      xVal = ((col + P.xStart) + rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5)) * P.fishMult;
      rSq = yVal * yVal + xVal * xVal;
      traced = rSq <= 1;
    }
    const double r = sqrt(rSq), theta = r * P.aperHalf, phi = atan2(-yVal, xVal), sTh = jf::sin(theta);
    o = mk(0, 0, 0);
    d = mk(sTh * jf::cos(phi), sTh * jf::sin(phi), -jf::cos(theta));
  } else if ((F & FT_CAMX) && P.cam == 2) {
    const double rayYOffset = P.H / 2.0, rayXOffset = P.W / 2.0;
    double rx, ry;
    if (n == 1) {
      ry = P.orthPerRow * (-1 * (row - rayYOffset));
      rx = P.orthPerCol * (col - rayXOffset);
    } else {
      const double yB = P.orthPerRow * ((-1 * (row - rayYOffset)) - .5), xB = P.orthPerCol * (col - rayXOffset - .5);
      ry = yB + (P.orthPerRow * rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5));
      rx = xB + (P.orthPerCol * rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5));
    }
    o = mk(rx, ry, 0);
    d = mk(0, 0, -1);
  } else if (dof) {
    double th = rng(P.seed, pixel, (uint32_t)s, 0, SITE_DOF_ANG, 0, 0, TWO_PI_F);
    V tt = nrmz(rot_axis(mk(0, 1, 0), mk(0, 0, -1), th));
    double mm = rng(P.seed, pixel, (uint32_t)s, 0, SITE_DOF_RAD, 0, 0, S.lensRadius);
    tt = mk(tt.x * mm, tt.y * mm, tt.z * mm);
    o = mk(tt.x + lc.x, tt.y + lc.y, tt.z + lc.z);
    d = sub(fpt, o);
  } else if (n == 1) {
    o = mk(0, 0, 0);
    d = mk(rayX, rayY, P.viewZ);
  } else {
    double ry = rayY + rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_Y, 0, -.5, .5);
    double rx = rayX + rng(P.seed, pixel, (uint32_t)s, 0, SITE_AA_X, 0, -.5, .5);
    o = mk(0, 0, 0);
    d = mk(rx, ry, P.viewZ);
  }
  return traced;
}

// one ray of one level: closest hit, then either a finished colour (miss: the background; a hit
// without children: its clamped local colour) or a frame with 1-2 child rays
struct WfOut {
  V c;         // finished colour (nch == 0)
  int nch;     // children spawned
  Child a, b;  // child A (or the only child), child B
  int sideA;   // 0: the first child is A; 1: it is B (phase 3: only the Fresnel reflection)
};
template <uint32_t F>
DEVI WfOut wf_shade(const SceneD& S, const Child& in, Key& k, WfNode& rec) {
  Counters ct;
  WfOut r;
  r.nch = 0;
  r.sideA = 0;
  WRay w;
  w.o = in.o; w.d = nrmz(in.d); w.d0 = w.d; w.stable = false; w.moved = false; w.ver = 0;  // myRay ctor
  k.node = in.node;
  Best b = closest<false, F, PACKET>(S, w, k, ct);
  rec.kind = 0;
  if (b.t == DMAX) {
    r.c = background<false, F>(S, w, ct);
    return r;
  }
  HitRec h = make_hit<F>(S, b, w, k);
  bool branch;
  FrameOf<F> Fr;
  Child a;
  V loc;
  const int nch = shade_node<false, F, false>(S, h, in, k, Fr, loc, a, branch, ct);  // every frame field
  if (nch == 0) {
    r.c = branch ? clampc(add(loc, mk(0, 0, 0))) : clampc(loc);
    return r;
  }
  rec.kind = 1;
  rec.local[0] = loc.x; rec.local[1] = loc.y; rec.local[2] = loc.z;
  rec.mat = Fr.mat;
  rec.phase = ((F & FT_TRANS) != 0) ? Fr.phase : 1;
  r.a = a;
  if constexpr ((F & FT_TRANS) != 0) {
    rec.mode = Fr.mode;
    rec.wa = Fr.wa;
    rec.wb = Fr.wb;
    rec.hasB = Fr.hasB;
    if (Fr.phase == 3) r.sideA = 1;
    if (Fr.phase == 1 && Fr.hasB) {  // the Fresnel reflection child, spawned here instead of after A returns
      r.b.o = Fr.org; r.b.d = Fr.dB; r.b.gen = Fr.gen + 1; r.b.node = Fr.node * 2 + 1;
      r.b.ktm = (Fr.mode == FM_SIMPLE) ? -1 : Fr.mat;
    }
  } else {
    rec.mode = FM_REFL;
    rec.hasB = 0;
  }
  r.nch = nch;
  return r;
}

// a node's colour from its children (trace_sample's fold, same operations in the same order)
template <uint32_t F>
DEVI V wf_fold(const SceneD& S, const WfNode& P) {
  const MatD& m = S.mat[P.mat];
  const V cA = mk(P.cA[0], P.cA[1], P.cA[2]), cB = mk(P.cB[0], P.cB[1], P.cB[2]);
  const V local = mk(P.local[0], P.local[1], P.local[2]);
  V acc;
  if ((F & FT_TRANS) == 0 || P.mode == FM_REFL) {
    const double* wA = m.kreflclr;
    acc = mk(0 + (wA[0] * cA.x), 0 + (wA[1] * cA.y), 0 + (wA[2] * cA.z));
  } else {
    V a0 = mk(0, 0, 0);
    bool haveA = false;
    if (P.phase == 1) {
      V wA;
      if (P.mode == FM_SIMPLE) { const double w = P.wa * m.ktrans; wA = mk(w, w, w); }
      else wA = mk(P.wa * m.permclr[0], P.wa * m.permclr[1], P.wa * m.permclr[2]);
      a0 = mk(0 + (wA.x * cA.x), 0 + (wA.y * cA.y), 0 + (wA.z * cA.z));
      haveA = true;
    }
    if (P.phase == 3 || (haveA && P.hasB)) {
      V wB;
      if (P.mode == FM_SIMPLE) { const double w = P.wb * m.krefl; wB = mk(w, w, w); }
      else wB = mk(P.wb * m.permclr[0], P.wb * m.permclr[1], P.wb * m.permclr[2]);
      acc = mk(a0.x + (wB.x * cB.x), a0.y + (wB.y * cB.y), a0.z + (wB.z * cB.z));
    } else {
      acc = a0;
    }
  }
  return clampc(add(local, acc));
}
DEVI void wf_put(double* dst, V c) { dst[0] = c.x; dst[1] = c.y; dst[2] = c.z; }
// A parent outside the previous level or a child past the queue's capacity would be an indexing bug:
// it is not written, and the launch's error word is set (render_wf returns RT_E_HIP for it).
DEVI void wf_deliver(WfNode* prev, int32_t nPrev, int32_t parent, V c, int* __restrict__ err) {
  if ((uint32_t)(parent >> 1) >= (uint32_t)nPrev) {
    atomicOr(err, 1);
    return;
  }
  WfNode& p = prev[parent >> 1];
  wf_put((parent & 1) ? p.cB : p.cA, c);
}

// children of a wave into the next level's queue: ballot + mbcnt prefix counts, one atomic add
DEVI void wf_emit(const WfOut& r, int32_t me, const Key& k, WfRay* __restrict__ qout, int* __restrict__ cntOut, int32_t qcap,
                  int* __restrict__ err) {
  const uint64_t b1 = __ballot(r.nch >= 1), b2 = __ballot(r.nch == 2);
  if (!(b1 | b2)) return;
  const uint32_t tot = (uint32_t)(__popcll(b1) + __popcll(b2));
  const int first = (int)__builtin_ctzll(__ballot(1));
  int base = 0;
  if ((int)__lane_id() == first) base = atomicAdd(cntOut, (int)tot);
  base = __builtin_amdgcn_readlane(base, first);
  const uint32_t below = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
  const uint32_t below2 = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b2, 0u));
  auto put = [&](int slot, const Child& c, int side) {
    if (slot >= qcap) {  // (at most two children per ray: the queue holds them all)
      atomicOr(err, 2);
      return;
    }
    WfRay& q = qout[slot];
    q.o[0] = c.o.x; q.o[1] = c.o.y; q.o[2] = c.o.z;
    q.d[0] = c.d.x; q.d[1] = c.d.y; q.d[2] = c.d.z;
    q.pixel = k.pixel; q.sample = k.sample; q.node = c.node; q.gen = c.gen; q.ktm = c.ktm;
    q.parent = (me << 1) | side;
  };
  if (r.nch >= 1) put(base + (int)below, r.a, r.sideA);
  if (r.nch == 2) put(base + __popcll(b1) + (int)below2, r.b, 1);
}

// level 0: the camera samples of `nunits` (tile, round) units starting at tile tile0
template <uint32_t F>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WF_WAVES)))
wf_camera_kernel(SceneD S, ParamsD P, int tile0, int rounds, WfNode* __restrict__ node0, double* __restrict__ scol,
                 uint8_t* __restrict__ straced, WfRay* __restrict__ qout, int* __restrict__ cntOut, int32_t qcap,
                 int* __restrict__ err) {
  const int lane = threadIdx.x;
  const int unit = blockIdx.x, tile = tile0 + unit / rounds, round = unit % rounds;
  const int me = unit * 64 + lane;
  const int ncols = (F & FT_PASS) ? (P.W + P.colStep - 1) / P.colStep : P.W;
  const int tilesX = (ncols + P.tw - 1) / P.tw;
  const PixGeo g = pix_geo<F>(lane, tile, tilesX, ncols, P);
  const int s = round * P.G + g.j;
  const bool dof = (F & FT_DOF) && S.dof && !((F & FT_CAMX) && P.cam != 0);
  Key k;
  k.seed = P.seed;
  k.tsite = SITE_TIME;
  k.pixel = (uint64_t)g.row * (uint64_t)P.W + (uint64_t)g.col;
  k.sample = (uint32_t)s;
  V fpt = mk(0, 0, 0), lc = mk(0, 0, 0);
  if (dof && g.valid) {  // shootMultiDpthOfFldRays (myScene.java:1386-1406), as render_kernel
    const double rayY = (-1 * (g.row - P.H / 2.0)), rayX = g.col - P.W / 2.0;
    lc = nrmz(mk(rayX, rayY, P.viewZ));
    const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    V ld = nrmz(nrmz(lc));
    V fo = xpt(I, mk(0, 0, 0)), fd = xvec(I, ld);
    V fN = mk(0, 0, 1);
    double pr = dot(fN, fd);
    double t = -(dot(fN, fo) + S.lensFocal) / pr;
    fpt = mk(fd.x * t + fo.x, fd.y * t + fo.y, fd.z * t + fo.z);
  }
  WfOut r;
  r.nch = 0;
  r.c = mk(0, 0, 0);
  bool traced = false;
  WfNode& rec = node0[me];
  rec.kind = 0;
  if (g.valid && s < P.spp) {
    V o, d;
    traced = wf_camera<F>(S, P, g, s, dof, fpt, lc, k.pixel, o, d);
    if (traced) {
      Child in;
      in.o = o; in.d = d; in.node = 1; in.gen = 0; in.ktm = -1;
      r = wf_shade<F>(S, in, k, rec);
    }
  }
  straced[me] = traced ? 1 : 0;
  if (r.nch == 0) wf_put(scol + 3 * (size_t)me, r.c);
  wf_emit(r, me, k, qout, cntOut, qcap, err);
}

// level L >= 1: every queued ray of the level
template <uint32_t F>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WF_WAVES)))
wf_level_kernel(SceneD S, ParamsD P, const WfRay* __restrict__ qin, const int* __restrict__ cntIn,
                WfNode* __restrict__ nodeL, WfNode* __restrict__ nodePrev, int32_t nPrev, WfRay* __restrict__ qout,
                int* __restrict__ cntOut, int32_t qcap, int* __restrict__ err) {
  const int me = blockIdx.x * 64 + threadIdx.x;
  if (blockIdx.x * 64 >= *cntIn) return;  // whole wave past the queue
  const bool live = me < *cntIn;
  WfOut r;
  r.nch = 0;
  Key k;
  k.seed = P.seed;
  k.tsite = SITE_TIME;
  k.pixel = 0;
  k.sample = 0;
  int32_t parent = 0;
  if (live) {
    const WfRay& q = qin[me];
    Child in;
    in.o = mk(q.o[0], q.o[1], q.o[2]); in.d = mk(q.d[0], q.d[1], q.d[2]);
    in.node = q.node; in.gen = q.gen; in.ktm = q.ktm;
    k.pixel = q.pixel; k.sample = q.sample;
    parent = q.parent;
    r = wf_shade<F>(S, in, k, nodeL[me]);
    if (r.nch == 0) wf_deliver(nodePrev, nPrev, parent, r.c, err);
    else nodeL[me].parent = parent;  // where this frame's fold delivers
  }
  wf_emit(r, me, k, qout, cntOut, qcap, err);
}

// fold of one level's frames into their parents (level 0: into the sample colours)
template <uint32_t F>
__global__ void __launch_bounds__(256) wf_fold_kernel(SceneD S, const WfNode* __restrict__ nodeL, const int* __restrict__ cnt,
                                                      int n0, WfNode* __restrict__ nodePrev, int32_t nPrev,
                                                      double* __restrict__ scol, int* __restrict__ err) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = cnt ? *cnt : n0;
  if (i >= n) return;
  const WfNode& P = nodeL[i];
  if (!P.kind) return;
  const V c = wf_fold<F>(S, P);
  if (nodePrev) wf_deliver(nodePrev, nPrev, P.parent, c, err);
  else wf_put(scol + 3 * (size_t)i, c);
}

// per-pixel sums of the chunk's samples in sample order, then render_kernel's epilogue
template <uint32_t F>
__global__ void __launch_bounds__(64) wf_final_kernel(ParamsD P, int tile0, int rounds, const double* __restrict__ scol,
                                                      const uint8_t* __restrict__ straced, float* __restrict__ rgb,
                                                      int32_t* __restrict__ argb, int dof) {
  const int lane = threadIdx.x;
  const int tile = tile0 + blockIdx.x;
  const int ncols = (F & FT_PASS) ? (P.W + P.colStep - 1) / P.colStep : P.W;
  const int tilesX = (ncols + P.tw - 1) / P.tw;
  const PixGeo g = pix_geo<F>(lane, tile, tilesX, ncols, P);
  if (!g.valid || g.j != 0) return;
  const int n = P.spp, G = P.G;
  double rs = 0, gs = 0, bs = 0;
  for (int s = 0; s < n; ++s) {
    const size_t slot = ((size_t)blockIdx.x * rounds + s / G) * 64 + g.pl * G + (s % G);
    if (n == 1 && !dof) {
      rs = scol[3 * slot]; gs = scol[3 * slot + 1]; bs = scol[3 * slot + 2];
    } else if (straced[slot]) {
      rs += scol[3 * slot]; gs += scol[3 * slot + 1]; bs += scol[3 * slot + 2];
    }
  }
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

}  // namespace dv
}  // namespace rt

namespace rt {
namespace dv {
// ---------------------------------------------------------------------------
// Sample waves (rt_render_pixels_device): the samples of a few listed pixels, ONE sample per wave
// (lane 0 of a 64-lane workgroup), each colour kept, then every pixel summed in sample order. A
// pixel's 16 or 64 samples run in parallel on as many SIMDs instead of sharing one wave, whose
// packet traversal walks the union of their paths: the multi-GPU split renders its heaviest tiles
// this way so that no single wave outlasts a rank's share of the frame. Same samples, same keys,
// same order of the per-pixel sum: the same pixels as render_kernel.
template <uint32_t F>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_RENDER_WAVES)))
sample_kernel(SceneD S, ParamsD P, const int32_t* __restrict__ pix, double* __restrict__ col, uint8_t* __restrict__ tr) {
  if (threadIdx.x != 0) return;
  const int b = blockIdx.x, i = b / P.spp, s = b % P.spp;
  const int px = pix[i];
  PixGeo g;
  g.row = px / P.W;
  g.col = px % P.W;
  g.valid = true;
  g.j = 0; g.pl = 0; g.ci = g.col; g.ri = g.row;
  const bool dof = (F & FT_DOF) && S.dof && !((F & FT_CAMX) && P.cam != 0);
  Key k;
  k.seed = P.seed;
  k.tsite = SITE_TIME;
  k.pixel = (uint64_t)g.row * (uint64_t)P.W + (uint64_t)g.col;
  k.sample = (uint32_t)s;
  V fpt = mk(0, 0, 0), lc = mk(0, 0, 0);
  if (dof) {  // shootMultiDpthOfFldRays (myScene.java:1386-1406), as render_kernel
    const double rayY = (-1 * (g.row - P.H / 2.0)), rayX = g.col - P.W / 2.0;
    lc = nrmz(mk(rayX, rayY, P.viewZ));
    const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    V ld = nrmz(nrmz(lc));
    V fo = xpt(I, mk(0, 0, 0)), fd = xvec(I, ld);
    V fN = mk(0, 0, 1);
    double pr = dot(fN, fd);
    double t = -(dot(fN, fo) + S.lensFocal) / pr;
    fpt = mk(fd.x * t + fo.x, fd.y * t + fo.y, fd.z * t + fo.z);
  }
  V o, d, c = mk(0, 0, 0);
  const bool traced = wf_camera<F>(S, P, g, s, dof, fpt, lc, k.pixel, o, d);
  if (traced) {
    Counters ct;
    c = trace_sample<false, F>(S, o, d, k, ct);
  }
  wf_put(col + 3 * (size_t)b, c);
  tr[b] = traced ? 1 : 0;
}
// the listed pixels' sums in sample order and render_kernel's epilogue (whole-frame layout)
__global__ void __launch_bounds__(256) pixel_sum_kernel(ParamsD P, const int32_t* __restrict__ pix, int npix,
                                                        const double* __restrict__ col, const uint8_t* __restrict__ tr,
                                                        float* __restrict__ rgb, int32_t* __restrict__ argb, int dof) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= npix) return;
  const int n = P.spp;
  double rs = 0, gs = 0, bs = 0;
  for (int s = 0; s < n; ++s) {
    const size_t b = (size_t)i * n + s;
    if (n == 1 && !dof) {
      rs = col[3 * b]; gs = col[3 * b + 1]; bs = col[3 * b + 2];
    } else if (tr[b]) {
      rs += col[3 * b]; gs += col[3 * b + 1]; bs += col[3 * b + 2];
    }
  }
  const V c = (n == 1 && !dof) ? mk(rs, gs, bs) : clampc(mk(rs / n, gs / n, bs / n));
  const size_t o = (size_t)pix[i];
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
}  // namespace dv
}  // namespace rt
