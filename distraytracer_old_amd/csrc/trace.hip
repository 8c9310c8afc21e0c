// C-ABI render entry points (include/distraytracer.h): scene upload, kernel
// variant dispatch, launches and the photon pre-pass driver. The kernels are in
// trace_kernels.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "rt_internal.h"
#include "trace_kernels.h"
#include "wavefront.h"
// ===========================================================================
// host side: device upload + C ABI
using namespace rt;

static thread_local std::string g_last_error;
int rt::set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_error(RT_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

static const int H_PERM[256] = {151,160,137,91,90,15,131,13,201,95,96,53,194,233,7,225,140,36,103,30,69,142,8,99,37,240,21,10,23,
  190,6,148,247,120,234,75,0,26,197,62,94,252,219,203,117,35,11,32,57,177,33,88,237,149,56,87,174,20,125,136,171,168,68,175,74,165,71,
  134,139,48,27,166,77,146,158,231,83,111,229,122,60,211,133,230,220,105,92,41,55,46,245,40,244,102,143,54,65,25,63,161,1,216,80,73,209,
  76,132,187,208,89,18,169,200,196,135,130,116,188,159,86,164,100,109,198,173,186,3,64,52,217,226,250,124,123,5,202,38,147,118,126,255,
  82,85,212,207,206,59,227,47,16,58,17,182,189,28,42,223,183,170,213,119,248,152,2,44,154,163,70,221,153,101,155,167,43,172,9,129,22,39,
  253,19,98,108,110,79,113,224,232,178,185,112,104,218,246,97,228,251,34,242,193,238,210,144,12,191,179,162,241,81,51,145,235,249,14,239,
  107,49,192,214,31,181,199,106,157,184,84,204,176,115,121,50,45,127,4,150,254,138,236,205,93,222,114,67,29,24,72,243,141,128,195,78,66,
  215,61,156,180};
static const int H_GRAD3[12][3] = {{1,1,0},{-1,1,0},{1,-1,0},{-1,-1,0},{1,0,1},{-1,0,1},{1,0,-1},{-1,0,-1},{0,1,1},{0,-1,1},{0,1,-1},{0,-1,-1}};

template <class T>
static int upload(rt_scene* s, const std::vector<T>& v, const T** out) {
  if (v.empty()) { *out = nullptr; return RT_OK; }
  void* p = nullptr;
  size_t bytes = v.size() * sizeof(T);
  HIPCHK(hipMalloc(&p, bytes));
  s->allocs.push_back(p);
  s->devBytes += bytes;
  HIPCHK(hipMemcpy(p, v.data(), bytes, hipMemcpyHostToDevice));
  *out = (const T*)p;
  return RT_OK;
}

// Conservative world-space bounds used to skip top-level entries a ray cannot hit
// (closest() / shadowed(), trace_kernels.h top_culled):
//  * implicit primitives (spheres, moving spheres, capped / hollow cylinders, rendered
//    boxes): the object-space box of the shape (a cylinder's y range widened by its 1e-7
//    acceptance slack), its 8 corners through the CTM;
//  * BVHs / lists (TOP_ACCEL): every member's world geometry -- triangles enlarged by the
//    reference's fat-edge acceptance (an inside test >= -1e-7 on unnormalised edge cross
//    products accepts points up to 1e-7 / |edge| outside an edge, myPlanarObject.java:165-175),
//    implicit members as above; lists holding quads, planes or instances get no bound.
// Each becomes the sphere around the world box, inflated by 1e-6 relative + absolute. A ray
// that misses it, or enters it beyond the current best hit / the shadow distance, cannot
// produce a hit the reference would keep.
static void box_union(double* mn, double* mx, const double* p) {
  for (int c = 0; c < 3; ++c) { mn[c] = std::min(mn[c], p[c]); mx[c] = std::max(mx[c], p[c]); }
}
static void xform_pt(const double* g, const double* p, double* w) {
  for (int r = 0; r < 3; ++r) w[r] = g[r * 4 + 0] * p[0] + g[r * 4 + 1] * p[1] + g[r * 4 + 2] * p[2] + g[r * 4 + 3];
}
// world box of an implicit primitive; false for other kinds
static bool implicit_world_box(const HostScene& h, const PrimD& P, int xf, double* wmn, double* wmx) {
  double mn[3], mx[3];
  switch (P.type) {
    case PT_SPHERE:
    case PT_MSPHERE:
      for (int c = 0; c < 3; ++c) {
        const double r = std::fabs(P.a[3 + c]);
        mn[c] = P.a[c] - r; mx[c] = P.a[c] + r;
        if (P.type == PT_MSPHERE) { mn[c] = std::min(mn[c], P.a[6 + c] - r); mx[c] = std::max(mx[c], P.a[6 + c] + r); }
      }
      break;
    case PT_CYL:
    case PT_HCYL: {
      const double rx = std::fabs(P.a[3]), rz = std::fabs(P.a[4]);
      mn[0] = P.a[0] - rx; mx[0] = P.a[0] + rx;
      mn[2] = P.a[2] - rz; mx[2] = P.a[2] + rz;
      mn[1] = std::min(P.a[7], P.a[6]) - 1e-6; mx[1] = std::max(P.a[7], P.a[6]) + 1e-6;
      break;
    }
    case PT_BOX:
      for (int c = 0; c < 3; ++c) { mn[c] = P.a[c]; mx[c] = P.a[3 + c]; }
      break;
    default:
      return false;
  }
  const double* g = h.xf[xf].g;
  for (int k = 0; k < 8; ++k) {
    const double p[3] = {(k & 1) ? mx[0] : mn[0], (k & 2) ? mx[1] : mn[1], (k & 4) ? mx[2] : mn[2]};
    double w[3];
    xform_pt(g, p, w);
    box_union(wmn, wmx, w);
  }
  return true;
}
// world box of a triangle with its fat-edge acceptance region: in the triangle's plane each
// edge line moves outward by 1e-7 / |edge| (plus slack); the enlarged triangle's corners are
// the intersections of adjacent moved lines. False when an angle is too acute to bound.
static bool tri_world_box(const HostScene& h, const TriD& T, double* wmn, double* wmx) {
  const double* v[3] = {T.v[0], T.v[1], T.v[2]};
  double e[3][3], len[3];
  for (int i = 0; i < 3; ++i) {
    const double* a = v[i];
    const double* b = v[(i + 1) % 3];
    for (int c = 0; c < 3; ++c) e[i][c] = b[c] - a[c];
    len[i] = std::sqrt(e[i][0] * e[i][0] + e[i][1] * e[i][1] + e[i][2] * e[i][2]);
    if (!(len[i] > 0) || !std::isfinite(len[i])) return false;
  }
  // corner i (at v[i], between edge i-1 and edge i, angle A): moving the two edge lines
  // outward by da, db moves their intersection by sqrt(da^2 + db^2 + 2 da db cos A) / sin A
  // <= (da + db) / sin A
  double grow = 0;
  for (int i = 0; i < 3; ++i) {
    const int ia = (i + 2) % 3;
    const double* ea = e[ia];  // into v[i]
    const double* eb = e[i];   // out of v[i]
    const double cosA = -(ea[0] * eb[0] + ea[1] * eb[1] + ea[2] * eb[2]) / (len[ia] * len[i]);
    const double sinA = std::sqrt(std::max(0.0, 1 - cosA * cosA));
    if (!(sinA > 1e-4)) return false;
    const double da = 1e-7 / len[ia] * 1.01 + 1e-12, db = 1e-7 / len[i] * 1.01 + 1e-12;
    grow = std::max(grow, (da + db) / sinA);
  }
  double mn[3], mx[3];
  for (int c = 0; c < 3; ++c) {
    mn[c] = std::min(v[0][c], std::min(v[1][c], v[2][c])) - grow;
    mx[c] = std::max(v[0][c], std::max(v[1][c], v[2][c])) + grow;
  }
  const double* g = h.xf[T.xf].g;
  for (int k = 0; k < 8; ++k) {
    const double p[3] = {(k & 1) ? mx[0] : mn[0], (k & 2) ? mx[1] : mn[1], (k & 4) ? mx[2] : mn[2]};
    double w[3];
    xform_pt(g, p, w);
    box_union(wmn, wmx, w);
  }
  return true;
}
// members of an accel: walk its node tree (rt_types.h child references)
static bool accel_world_box(const HostScene& h, const AccelD& A, double* wmn, double* wmx) {
  std::vector<int32_t> stack{A.root};
  while (!stack.empty()) {
    const int32_t r = stack.back();
    stack.pop_back();
    if (r >= 0) {
      stack.push_back(h.node[r].left);
      stack.push_back(h.node[r].right);
      continue;
    }
    const int32_t c = ~r;
    int32_t start, count;
    const bool run = (c & LEAF_RUN_FLAG) != 0;
    if (run) { start = (c >> 5) & LEAF_RUN_MAXSTART; count = c & 31; }
    else { start = h.leaf[c].start; count = h.leaf[c].count; }
    for (int i = 0; i < count; ++i) {
      const int32_t m = run ? start + i : h.member[start + i];
      if (m >= 0) {
        if (!tri_world_box(h, h.tri[m], wmn, wmx)) return false;
      } else {
        const PrimD& P = h.prim[~m];
        if (!implicit_world_box(h, P, P.xf, wmn, wmx)) return false;  // quads, planes, instances
      }
    }
  }
  return true;
}
static std::vector<double> top_bounds(const HostScene& h) {
  std::vector<double> b(4 * h.top.size(), -1.0);
  for (size_t i = 0; i < h.top.size(); ++i) {
    const TopD& t = h.top[i];
    double wmn[3] = {1e300, 1e300, 1e300}, wmx[3] = {-1e300, -1e300, -1e300};
    if (t.kind == TOP_PRIM) {
      if (!implicit_world_box(h, h.prim[t.idx], t.xf, wmn, wmx)) continue;  // quads / planes: never culled
    } else if (t.kind == TOP_ACCEL) {
      if (!accel_world_box(h, h.accel[t.idx], wmn, wmx)) continue;
    } else {
      continue;  // top-level triangles, instances
    }
    double c[3], hd2 = 0, cn = 0;
    for (int r = 0; r < 3; ++r) {
      c[r] = 0.5 * (wmn[r] + wmx[r]);
      const double e = 0.5 * (wmx[r] - wmn[r]);
      hd2 += e * e;
      cn += c[r] * c[r];
    }
    const double R = std::sqrt(hd2) * (1 + 1e-6) + 1e-6 * (1 + std::sqrt(cn));
    if (!std::isfinite(R) || !std::isfinite(cn)) continue;
    b[4 * i + 0] = c[0]; b[4 * i + 1] = c[1]; b[4 * i + 2] = c[2]; b[4 * i + 3] = R;
  }
  return b;
}

// World planes of the top-level quads / planes / triangles (after the 4 * ntop sphere bounds, 8 doubles per
// entry: orientation A's and B's plane as unit normal + offset, zero normal = none). A hit of
// orientation A lies on N_A . x + d_A = 0 in object space (trace_device.h planar_test), so on
// n . y + d = 0 in world space with n = A^-T N_A, d = d_A - n . b (y = A x + b, the entry's CTM).
// The wave-level shadow cull (trace_kernels.h step_cands) skips the entry for a wave whose shadow
// segments all stay strictly on one side of both planes.
static std::vector<double> top_planes(const HostScene& h) {
  std::vector<double> b(8 * h.top.size(), 0.0);
  for (size_t i = 0; i < h.top.size(); ++i) {
    const TopD& t = h.top[i];
    double NA[3], NB[3], DA, DB;
    if (t.kind == TOP_PRIM && (h.prim[t.idx].type == PT_QUAD || h.prim[t.idx].type == PT_PLANE)) {
      const PrimD& P = h.prim[t.idx];
      for (int c = 0; c < 3; ++c) { NA[c] = P.a[12 + c]; NB[c] = P.a[15 + c]; }
      DA = P.a[18]; DB = P.a[19];
    } else if (t.kind == TOP_TRI) {  // tri_test: orientation B is -n with dB
      const TriD& T = h.tri[t.idx];
      for (int c = 0; c < 3; ++c) { NA[c] = T.n[c]; NB[c] = -T.n[c]; }
      DA = T.dA; DB = T.dB;
    } else {
      continue;
    }
    const double* g = h.xf[t.xf].g;
    const double* inv = h.xf[t.xf].inv;
    for (int o = 0; o < 2; ++o) {
      const double* N = o ? NB : NA;
      const double D = o ? DB : DA;
      double n[3];
      for (int c = 0; c < 3; ++c) n[c] = inv[0 * 4 + c] * N[0] + inv[1 * 4 + c] * N[1] + inv[2 * 4 + c] * N[2];
      const double d = D - (n[0] * g[3] + n[1] * g[7] + n[2] * g[11]);
      const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      if (!(len > 0) || !std::isfinite(len) || !std::isfinite(d)) { std::fill(&b[8 * i], &b[8 * i] + 8, 0.0); break; }
      for (int c = 0; c < 3; ++c) b[8 * i + 4 * o + c] = n[c] / len;
      b[8 * i + 4 * o + 3] = d / len;
    }
  }
  return b;
}

static int upload_scene(rt_scene* s) {
  HostScene& h = s->hs;
  SceneD& d = s->dev;
  int rc;
  if ((rc = upload(s, h.xf, &d.xf)) || (rc = upload(s, h.tri, &d.tri)) || (rc = upload(s, h.prim, &d.prim)) ||
      (rc = upload(s, h.node, &d.node)) || (rc = upload(s, h.leaf, &d.leaf)) || (rc = upload(s, h.member, &d.member)) ||
      (rc = upload(s, h.accel, &d.accel)) || (rc = upload(s, h.top, &d.top)) || (rc = upload(s, h.mat, &d.mat)) ||
      (rc = upload(s, h.light, &d.light)) || (rc = upload(s, h.tex, &d.tex)) || (rc = upload(s, h.texel, &d.texel)))
    return rc;
  {  // fp32 node boxes (trace_kernels.h box32): coordinates rounded to nearest, bounds rounded up
    auto f32 = [](double x) { return std::fabs(x) <= 3.0e38 ? (float)x : (x < 0 ? -INFINITY : INFINITY); };
    auto f32_up = [](double x) {  // >= x >= 0 (inf when it does not fit)
      const double u = x * (1 + 0x1p-20);
      return (u >= 0 && u <= 3.0e38) ? (float)u : INFINITY;
    };
    std::vector<NodeF> nf(h.node.size());
    for (size_t i = 0; i < h.node.size(); ++i) {
      NodeD& n = h.node[i];
      const double* src[4] = {n.lmin, n.lmax, n.rmin, n.rmax};
      double mag = 0;
      for (int q = 0; q < 4; ++q)
        for (int c = 0; c < 3; ++c) {
          nf[i].b[3 * q + c] = f32(src[q][c]);
          mag = std::max(mag, std::fabs(src[q][c]));
        }
      nf[i].mag = std::isfinite(mag) ? f32_up(mag) : INFINITY;
      const double sl = node_slack(n, 0), sr = node_slack(n, 1);  // set for nearest-first accels only
      nf[i].sl = std::isfinite(sl) && sl >= 0 ? f32_up(sl) : INFINITY;
      nf[i].sr = std::isfinite(sr) && sr >= 0 ? f32_up(sr) : INFINITY;
      nf[i].pad = 0;
    }
    if ((rc = upload(s, nf, &d.nodeF))) return rc;
    // fp32 edge records of the triangles (trace_kernels.h tri_f32_out)
    std::vector<TriF> tf(h.tri.size());
    for (size_t i = 0; i < h.tri.size(); ++i) {
      const TriD& t = h.tri[i];
      TriF& r = tf[i];
      double mmax = 0, tm = std::fabs(t.dA);
      bool fin = std::isfinite(t.dA);
      for (int j = 0; j < 3; ++j) {
        const double* a = t.v[j];
        const double* b = t.v[(j + 2) % 3];
        const double e[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
        const double m[3] = {e[1] * t.n[2] - e[2] * t.n[1], e[2] * t.n[0] - e[0] * t.n[2], e[0] * t.n[1] - e[1] * t.n[0]};
        const double c = a[0] * m[0] + a[1] * m[1] + a[2] * m[2];
        for (int q = 0; q < 3; ++q) { r.m[j][q] = f32(m[q]); fin = fin && std::isfinite(m[q]) && std::isfinite(a[q]); }
        r.c[j] = f32(c);
        r.n[j] = f32(t.n[j]);
        fin = fin && std::isfinite(c) && std::isfinite(t.n[j]);
        mmax = std::max(mmax, std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]));
        tm = std::max(tm, std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]));
      }
      const double nmag = std::sqrt(t.n[0] * t.n[0] + t.n[1] * t.n[1] + t.n[2] * t.n[2]);
      r.d = f32(t.dA);
      r.k = fin && std::isfinite(mmax) && std::isfinite(nmag) ? f32_up(0x1p-17 * mmax * std::max(1.0, nmag)) : INFINITY;
      r.tm = std::isfinite(tm) ? f32_up(tm) : INFINITY;
      r.pad[0] = r.pad[1] = 0;
      if (!std::isfinite(r.tm)) r.k = INFINITY;
    }
    if ((rc = upload(s, tf, &d.triF))) return rc;
  }
  d.triUV = nullptr;
  {  // triangle UVs only matter for image-textured triangles
    bool need = false;
    for (const TriD& t : h.tri) need = need || h.mat[t.mat].tex == RT_TEX_IMAGE;
    if (need && (rc = upload(s, h.triUV, &d.triUV))) return rc;
  }
  d.ntop = (int)h.top.size();
  {
    std::vector<double> tb = top_bounds(h), none(tb.size(), -1.0);
    const std::vector<double> tp = top_planes(h);
    tb.insert(tb.end(), tp.begin(), tp.end());
    none.insert(none.end(), tp.size(), 0.0);
    if ((rc = upload(s, tb, &d.topBound)) || (rc = upload(s, none, &s->noCullBound))) return rc;
  }
  d.nlight = (int)h.light.size();
  d.pnode = nullptr;
  d.ppos = d.ppwr = nullptr;
  d.nphoton = 0;
  d.photonRoot = 0;
  d.photonK = h.photonK;
  d.knnU16Max = 65535;  // DISTRAYTRACER_KNN_U16_MAX lowers it: a test of the u32 fallback
  if (const char* e = std::getenv("DISTRAYTRACER_KNN_U16_MAX")) d.knnU16Max = std::max(0, std::min(65535, std::atoi(e)));
  d.photonMaxD2 = h.photonMaxD2;
  for (int c = 0; c < 3; ++c) d.bg[c] = h.bg[c];
  d.bkgTex = h.bkgTex;
  for (int c = 0; c < 4; ++c) d.sky[c] = h.sky[c];
  d.dof = h.dof;
  d.lensRadius = h.lensRadius;
  d.lensFocal = h.lensFocal;
  d.numRays = 8;  // myScene.numRays
  // qdiv (trace_device.h) is exact only for box coordinates 0 or in [2^-200, 2^200]
  auto in_range = [](const double* c, int n) {
    for (int i = 0; i < n; ++i) {
      double a = std::fabs(c[i]);
      if (!(c[i] == 0 || (a >= 0x1p-200 && a <= 0x1p200))) return false;
    }
    return true;
  };
  bool ok = true;
  for (const NodeD& n : h.node) ok = ok && in_range(n.lmin, 3) && in_range(n.lmax, 3) && in_range(n.rmin, 3) && in_range(n.rmax, 3);
  for (const AccelD& a : h.accel) ok = ok && in_range(a.bmin, 3) && in_range(a.bmax, 3);
  d.fastSlab = ok ? SCENE_FAST_SLAB : 0;
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dv::c_perm), H_PERM, sizeof(H_PERM)));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dv::c_grad3), H_GRAD3, sizeof(H_GRAD3)));
  void* cnt = nullptr;
  HIPCHK(hipMalloc(&cnt, sizeof(unsigned long long) * RT_ST_N));
  s->allocs.push_back(cnt);
  s->counters = cnt;
  return RT_OK;
}

int rt_upload_photons(rt_scene* s) {  // after the host photon-map build (csrc/photon.cpp)
  HostScene& h = s->hs;
  HIPCHK(hipSetDevice(s->device));
  int rc;
  if ((rc = upload(s, h.pnode, &s->dev.pnode)) || (rc = upload(s, h.ppos, &s->dev.ppos)) ||
      (rc = upload(s, h.ppwr, &s->dev.ppwr)))
    return rc;
  s->dev.nphoton = (int)h.nphoton;
  s->dev.photonRoot = h.photonRoot;
  s->photonsUploaded = true;
  return RT_OK;
}

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_last_error.c_str(); }

int rt_device_count(int* count) {
  if (!count) return set_error(RT_E_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out) {
  if (!desc || !out) return set_error(RT_E_INVALID, "rt_scene_create: null argument");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(RT_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return set_error(RT_E_INVALID, "device ordinal out of range");
  rt_scene* s = new rt_scene();
  s->device = device;
  int rc = build_host_scene(desc, s->hs);
  if (rc == RT_OK) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) rc = set_error(RT_E_HIP, hipGetErrorString(e));
    else rc = upload_scene(s);
  }
  if (rc != RT_OK) {
    rt_scene_destroy(s);
    return rc;
  }
  *out = s;
  return RT_OK;
}

int rt_scene_info(const rt_scene* s, int64_t* info, int n) {
  if (!s || !info) return set_error(RT_E_INVALID, "null argument");
  const HostScene& h = s->hs;
  int64_t v[14] = {(int64_t)h.top.size(), (int64_t)h.light.size(), h.bvhInternal, h.bvhLeaves, h.bvhDepth,
                   h.bvhPrims, h.nprims, h.rpp, (int64_t)s->devBytes, (int64_t)h.tri.size(),
                   (int64_t)h.nphoton, (int64_t)h.mat.size(), h.photonMode, h.photonCount};
  for (int i = 0; i < n && i < 14; ++i) info[i] = v[i];
  return RT_OK;
}

int rt_scene_photons(const rt_scene* s, double* pos, double* pwr, int64_t n, int64_t* count) {
  if (!s || !count) return set_error(RT_E_INVALID, "null argument");
  const HostScene& h = s->hs;
  *count = h.nphoton;
  if (n > 0 && (!pos || !pwr)) return set_error(RT_E_INVALID, "null photon buffers");
  const int64_t m = std::min<int64_t>(n, h.nphoton);
  if (m > 0) {
    std::memcpy(pos, h.photonListPos.data(), sizeof(double) * 3 * m);
    std::memcpy(pwr, h.photonListPwr.data(), sizeof(double) * 3 * m);
  }
  return RT_OK;
}

void rt_scene_destroy(rt_scene* s) {
  if (!s) return;
  if (!s->allocs.empty() || s->stream || s->outRgb || s->outArgb || !s->tileLists.empty() || s->stage || s->wf[rt_scene::WF_CNT] || s->smpCol) {
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize((hipStream_t)s->stream);
    for (void* p : s->allocs) (void)hipFree(p);
    for (auto& e : s->schedules)
      if (e.measured) (void)hipEventDestroy((hipEvent_t)e.measured);
    (void)hipFree(s->outRgb);
    (void)hipFree(s->outArgb);
    for (auto& t : s->tileLists) (void)hipFree(t.dev);
    for (void* p : s->wf) (void)hipFree(p);
    (void)hipFree(s->smpCol);
    (void)hipFree(s->smpTr);
    if (s->stage) (void)hipHostFree(s->stage);
    if (s->stream) (void)hipStreamDestroy((hipStream_t)s->stream);
  }
  delete s;
}

}  // extern "C"

static int make_params(rt_scene* s, const rt_render_params* p, ParamsD& P) {
  if (!s || !p) return set_error(RT_E_INVALID, "null argument");
  if (p->width <= 0 || p->height <= 0) return set_error(RT_E_INVALID, "bad image size");
  int row1 = p->row1 <= 0 ? p->height : p->row1;
  int step = p->row_step <= 1 ? 1 : p->row_step;
  if (p->row0 < 0 || p->row0 >= row1 || row1 > p->height) return set_error(RT_E_INVALID, "bad row range");
  P.W = p->width;
  P.H = p->height;
  P.spp = p->spp > 0 ? p->spp : s->hs.rpp;
  if (P.spp <= 0) return set_error(RT_E_INVALID, "rays_per_pixel is 0 (scene has no fov/rays_per_pixel; Q26)");
  // the compacted shadow rays hand a shading lane's RNG key to another lane packed in 64 bits
  // (dv::key_pack): pixel index < 2^32, sample < 2^20
  if ((p->flags & RT_RENDER_SHCOMPACT) && ((int64_t)P.W * P.H > (int64_t)UINT32_MAX || P.spp >= (1 << 20)))
    return set_error(RT_E_INVALID, "RT_RENDER_SHCOMPACT: image larger than 2^32 pixels or spp >= 2^20");
  const int band = p->row_band <= 1 ? 1 : p->row_band;
  P.row0 = p->row0;
  P.rowStep = step;
  P.band = band;
  {  // rows row0 + k*step*band + j (0 <= j < band) below row1
    const int span = row1 - p->row0, period = step * band;
    const int full = span / period, rest = span % period;
    P.nrows = full * band + std::min(rest, band);
  }
  P.seed = p->seed;
  // wave layout (render_kernel): G = largest power of two <= min(spp, 64) sample lanes per pixel
  int G = 1;
#ifndef RT_MAX_G
#define RT_MAX_G 64
#endif
  while (G * 2 <= P.spp && G * 2 <= RT_MAX_G) G *= 2;
  // RT_RENDER_PIXEL_WAVES: one pixel per wave (64 sample lanes, those past spp idle) -- the same
  // samples in the same order per pixel, so the same image; the multi-GPU split renders its
  // heaviest tiles this way (their 2 x 2 pixels in four waves at once)
  if (p->flags & RT_RENDER_PIXEL_WAVES) {
    // (at spp = 1 the kernel's one-sample path keeps the colour as traced; the 64-lane layout would
    // sum it from 0, turning -0.0 into +0.0)
    if (P.spp < 2) return set_error(RT_E_INVALID, "RT_RENDER_PIXEL_WAVES needs spp >= 2");
    G = 64;
  }
  static const int TW[7] = {8, 8, 4, 4, 2, 2, 1};  // pixels per wave 64, 32, ..., 1 as tw x th
  int lg = 0;
  while ((1 << lg) < G) ++lg;
  P.G = G;
  P.tw = TW[lg];
  P.th = (64 / G) / P.tw;
  P.order = nullptr;
  P.tcost = nullptr;
  // myFOVScene.setSceneParams (myScene.java:1367-1381) at the requested resolution
  double fov = s->hs.fov, fovRad = M_PI * fov / 180.0;
  if (std::fabs(fov - 180) < .001) fovRad -= .0001;
  P.viewZ = -1 * (std::max(P.H, P.W) / 2.0) / std::tan(fovRad / 2);
  // myFishEyeScene / myOrthoScene constants (setImageSize :780-792, setSceneParams :1556-1560, :1683-1688)
  P.cam = s->hs.camera;
  P.colStep = 1;
  {
    const double maxDim = std::max(P.H, P.W), rayYOffset = P.H / 2.0, rayXOffset = P.W / 2.0;
    P.yStart = ((maxDim - P.H) / 2.0) - rayYOffset;
    P.xStart = ((maxDim - P.W) / 2.0) - rayXOffset;
    P.fishMult = 2.0 / maxDim;
    P.aperHalf = (M_PI * s->hs.cameraParam[0] / 180.0) / 2.0;
    const double div = std::min(P.W, P.H);  // the reference divides by the applet's (= image) size
    P.orthPerRow = s->hs.cameraParam[1] / div;
    P.orthPerCol = s->hs.cameraParam[0] / div;
  }
  if (s->hs.photonMode && !s->photonsUploaded) {
    int rc = rt_photons_build(s, p->seed);
    if (rc) return rc;
  }
  return RT_OK;
}

// scene feature mask (dv::FT_*): which code paths the scene can reach
static uint32_t scene_features(const HostScene& h) {
  uint32_t f = 0;
  if (!h.prim.empty()) f |= dv::FT_PRIM;
  for (const PrimD& q : h.prim)
    if (q.type == PT_INST) { f |= dv::FT_INST; break; }
  if (h.bkgTex >= 0) f |= dv::FT_TEX;
  if (h.photonMode) f |= dv::FT_PHOTON;
  if (h.dof) f |= dv::FT_DOF;
  if (h.camera != RT_CAMERA_FOV) f |= dv::FT_CAMX;
  for (const MatD& m : h.mat) {
    if (m.tex != 0) f |= dv::FT_TEX;
    if (m.tex == 5) f |= dv::FT_CELL;
    if (m.usePhotonMap) f |= dv::FT_PHOTON;
    if (m.ktrans > 0 || m.perm > 0.0) f |= dv::FT_TRANS;
  }
  for (const LightD& l : h.light)
    if (l.type != 0) f |= dv::FT_LIGHTX;
  return f;
}

typedef void (*RenderFn)(SceneD, ParamsD, float*, int32_t*, unsigned long long*);
struct Variant {
  uint32_t mask;
  RenderFn fn;
};
// smallest first; the first variant whose mask covers the scene's features runs
static const Variant kVariants[] = {
    {0u, dv::render_kernel<false, 0u>},
    {dv::FT_PRIM, dv::render_kernel<false, dv::FT_PRIM>},
    {dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX,
     dv::render_kernel<false, dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX>},
    {dv::FT_PRIM | dv::FT_TRANS | dv::FT_PHOTON | dv::FT_LIGHTX,
     dv::render_kernel<false, dv::FT_PRIM | dv::FT_TRANS | dv::FT_PHOTON | dv::FT_LIGHTX>},
    {dv::FT_PRIM | dv::FT_INST | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX,
     dv::render_kernel<false, dv::FT_PRIM | dv::FT_INST | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX>},
    {dv::FT_ALL, dv::render_kernel<false, dv::FT_ALL>},
};

// RT_RENDER_SHCOMPACT: the same variants with the wave's shadow rays traced compacted
// (render_kernel<..., true>); the ones the benchmark configs run, and the generic one
static const Variant kVariantsShc[] = {
    {0u, dv::render_kernel<false, 0u, true>},
    {dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX,
     dv::render_kernel<false, dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX, true>},
    {dv::FT_PRIM | dv::FT_TRANS | dv::FT_PHOTON | dv::FT_LIGHTX,
     dv::render_kernel<false, dv::FT_PRIM | dv::FT_TRANS | dv::FT_PHOTON | dv::FT_LIGHTX, true>},
    {dv::FT_ALL, dv::render_kernel<false, dv::FT_ALL, true>},
};

static RenderFn pick_variant(const HostScene& h, uint32_t flags) {
  uint32_t f = (flags & RT_RENDER_GENERIC) ? (uint32_t)dv::FT_ALL : scene_features(h);
  if (flags & RT_RENDER_SHCOMPACT) {
    for (const Variant& v : kVariantsShc)
      if ((f & ~v.mask) == 0) return v.fn;
  }
  for (const Variant& v : kVariants)
    if ((f & ~v.mask) == 0) return v.fn;
  return dv::render_kernel<false, dv::FT_ALL>;
}
// the feature mask of the variant pick_variant launches (without RT_RENDER_SHCOMPACT)
static uint32_t variant_mask(const HostScene& h, uint32_t flags) {
  const uint32_t f = (flags & RT_RENDER_GENERIC) ? (uint32_t)dv::FT_ALL : scene_features(h);
  for (const Variant& v : kVariants)
    if ((f & ~v.mask) == 0) return v.mask;
  return dv::FT_ALL;
}

// Instrumented (counting) instantiations of the timed variants the benchmark configs run -- C3's
// (triangles only: nearest-first BVH traversal compiled in), C4's and C5's -- so the counted record
// loads are the ones the timed kernel issues (bench.py's roofline numerator); other scenes count
// with the all-features kernel.
static const Variant kCountVariants[] = {
    {0u, dv::render_kernel<true, 0u>},
    {dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX,
     dv::render_kernel<true, dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX>},
    {dv::F_C5, dv::render_kernel<true, dv::F_C5>},
    {dv::FT_ALL, dv::render_kernel<true, dv::FT_ALL>},
};
static const Variant& count_variant(const HostScene& h, uint32_t flags) {
  const uint32_t m = (flags & RT_RENDER_SHCOMPACT) ? (uint32_t)dv::FT_ALL : variant_mask(h, flags);
  for (const Variant& v : kCountVariants)
    if (v.mask == m) return v;
  return kCountVariants[sizeof(kCountVariants) / sizeof(kCountVariants[0]) - 1];
}

// Dispatch schedule: tiles sorted by cost, longest first, so the long tiles do not end
// up in the tail of the launch (matters most for the small per-GPU launches of a
// multi-GPU frame). Per tile layout: the first render orders tiles by a probe (one
// un-jittered camera ray per tile, its counted work); the first plain render with that
// order also records every wave's duration (tcost), and the next render re-sorts the
// tiles by those measured times -- the same frame's real cost, far better than one probe
// ray (the probe's tail at N = 8 was 150-340 us of a ~0.9 ms launch). Only the ORDER in
// which tiles are dispatched depends on it, never a pixel. The probe, the read-back and
// the sorts run synchronously, once per layout.
#ifndef RT_XCD_HASH
#define RT_XCD_HASH 0
#endif
static int sort_tiles(rt_scene::TileSchedule& e, hipStream_t st) {
  std::vector<uint32_t> cost(e.ntiles);
  hipError_t r = hipStreamSynchronize(st);
  // the measuring launch may have run on another stream (rt_render's own vs a caller's
  // rt_render_device stream): wait for it before reading its wave times
  if (r == hipSuccess && e.measured) r = hipEventSynchronize((hipEvent_t)e.measured);
  if (r == hipSuccess) r = hipMemcpy(cost.data(), e.cost, sizeof(uint32_t) * e.ntiles, hipMemcpyDeviceToHost);
  if (r != hipSuccess) return set_error(RT_E_HIP, std::string("tile schedule: ") + hipGetErrorString(r));
  // sort key: cost in quarter-octave buckets; tiles of one bucket keep row-major order, so
  // waves running at the same time stay spatially close (shared cache lines) while the
  // order stays longest-first to within 19 %. A counting sort over the buckets (stable, O(n)):
  // C4's 1 M tiles sort in a few ms, where std::stable_sort took ~100 ms of the first frames.
  constexpr int NB = 4 * 32 + 1;  // bucket 0: cost 0; bucket 1 + floor(4 log2 c) for c >= 1
  std::vector<uint8_t> key(e.ntiles);
  int hist[NB] = {0};
  for (int i = 0; i < e.ntiles; ++i) {
    const int k = cost_bucket(cost[i]);
    key[i] = (uint8_t)k;
    hist[k]++;
  }
  int start[NB];
  for (int k = NB - 1, acc = 0; k >= 0; --k) { start[k] = acc; acc += hist[k]; }  // longest first
  std::vector<int32_t> order(e.ntiles);
  for (int i = 0; i < e.ntiles; ++i) order[start[key[i]]++] = i;
#if RT_XCD_HASH > 0
  // XCD-aware deal (experiment): blocks b and b + 8 share an XCD and its L2 (MI355X_MICROARCH.md).
  // Superblocks of RT_XCD_HASH x RT_XCD_HASH tiles are hashed to one of 8 lists, each keeping the
  // longest-first order; dispatch position p takes the next tile of list p % 8, so neighbouring tiles
  // run on one XCD while every XCD sees the same mix of costs. An empty list's positions take the
  // longest remaining list's next tile.
  if (e.tilesX > 0) {
    constexpr int SB = RT_XCD_HASH;
    std::vector<int32_t> lists[8];
    for (int i = 0; i < e.ntiles; ++i) {
      const int t = order[i], sx = (t % e.tilesX) / SB, sy = (t / e.tilesX) / SB;
      const uint32_t h = ((uint32_t)sx * 73856093u) ^ ((uint32_t)sy * 19349663u);
      lists[(h ^ (h >> 7) ^ (h >> 13)) & 7].push_back(t);
    }
    size_t pos[8] = {0};
    for (int p = 0; p < e.ntiles; ++p) {
      int x = p & 7;
      if (pos[x] == lists[x].size()) {
        size_t best = 0;
        for (int y = 0; y < 8; ++y)
          if (lists[y].size() - pos[y] > best) { best = lists[y].size() - pos[y]; x = y; }
      }
      order[p] = lists[x][pos[x]++];
    }
  }
#endif
  HIPCHK(hipMemcpy(e.order, order.data(), sizeof(int32_t) * e.ntiles, hipMemcpyHostToDevice));
  return RT_OK;
}

static int schedule(rt_scene* s, ParamsD& P, bool count, hipStream_t st) {
  P.order = nullptr;
  P.tcost = nullptr;
  if (P.nrows * (int64_t)((P.W + P.colStep - 1) / P.colStep) < (1 << 16)) return RT_OK;  // small renders: row-major
  char key[160];
  std::snprintf(key, sizeof(key), "%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%.17g", P.W, P.H, P.row0, P.nrows, P.rowStep, P.band,
                P.colStep, P.tw, P.th, P.G, P.viewZ);
  rt_scene::TileSchedule* e = nullptr;
  for (auto& x : s->schedules)
    if (x.key == key) { e = &x; break; }
  if (!e) {
    const int ncols = (P.W + P.colStep - 1) / P.colStep;
    const int tilesX = (ncols + P.tw - 1) / P.tw, ntiles = tilesX * ((P.nrows + P.th - 1) / P.th);
    uint32_t* d_cost = nullptr;
    int32_t* d_order = nullptr;
    HIPCHK(hipMalloc(&d_cost, sizeof(uint32_t) * ntiles));
    s->allocs.push_back(d_cost);
    HIPCHK(hipMalloc(&d_order, sizeof(int32_t) * ntiles));
    s->allocs.push_back(d_order);
    hipLaunchKernelGGL((dv::probe_kernel<dv::FT_ALL>), dim3((ntiles + 63) / 64), dim3(64), dv::LDS_BYTES, st, s->dev,
                       P, d_cost, ntiles);
    HIPCHK(hipGetLastError());
    s->schedules.push_back({key, d_order, d_cost, ntiles, 0});
    s->schedules.back().tilesX = tilesX;
    e = &s->schedules.back();
    int rc = sort_tiles(*e, st);
    if (rc) return rc;
  } else if (e->state == 1) {  // the previous render measured its waves: order by those times
    int rc = sort_tiles(*e, st);
    if (rc) return rc;
    e->state = 2;
  }
  if (e->state == 0 && !count) {  // measure this (plain) render's waves
    P.tcost = e->cost;
    e->state = 1;
  }
  P.order = e->order;
  return RT_OK;
}

// ---------------------------------------------------------------------------
// RT_RENDER_WAVEFRONT (wavefront.h): chunks of (tile, sample round) units, each traced level by
// level -- one launch per generation of the shading tree over its compacted ray queue, the count of
// the next level read back in between -- then folded bottom up and summed per pixel.
#ifndef RT_WF_CHUNK
#define RT_WF_CHUNK (1 << 24)  // camera samples per chunk
#endif
static int wf_grow(rt_scene* s, int i, size_t bytes) {
  if (s->wfCap[i] >= bytes) return RT_OK;
  (void)hipFree(s->wf[i]);
  s->wf[i] = nullptr;
  s->wfCap[i] = 0;
  HIPCHK(hipMalloc(&s->wf[i], bytes));
  s->wfCap[i] = bytes;
  return RT_OK;
}
template <uint32_t F>
static int render_wf(rt_scene* s, const SceneD& sd, const ParamsD& P, float* d_rgb, int32_t* d_argb, hipStream_t st) {
  using dv::WfNode;
  using dv::WfRay;
  const int ncols = P.W, tilesX = (ncols + P.tw - 1) / P.tw, ntiles = tilesX * ((P.nrows + P.th - 1) / P.th);
  const int rounds = (P.spp + P.G - 1) / P.G;
  long chunkSamples = RT_WF_CHUNK;
  if (const char* e = std::getenv("DISTRAYTRACER_WF_CHUNK")) chunkSamples = std::max(64L, std::atol(e));  // testing knob
  const int chunk = std::max(1, std::min(ntiles, (int)(chunkSamples / (64L * rounds))));
  const size_t slots = (size_t)chunk * rounds * 64;
  int rc;
  typedef rt_scene R;
  if ((rc = wf_grow(s, R::WF_NODE0, slots * sizeof(WfNode))) || (rc = wf_grow(s, R::WF_SCOL, slots * 3 * sizeof(double))) ||
      (rc = wf_grow(s, R::WF_TRACED, slots)) || (rc = wf_grow(s, R::WF_CNT, 16 * sizeof(int))) ||
      (rc = wf_grow(s, R::WF_Q1, 2 * slots * sizeof(WfRay))))
    return rc;
  const int dof = ((F & dv::FT_DOF) && sd.dof && !((F & dv::FT_CAMX) && P.cam != 0)) ? 1 : 0;
  // queue capacity divisor: a testing knob (DISTRAYTRACER_WF_QCAP_DIV, default 1) that undersizes the
  // queues so that the device's overflow guard, and its error word, are exercised
  int qdiv = 1;
  if (const char* e = std::getenv("DISTRAYTRACER_WF_QCAP_DIV")) qdiv = std::max(1, std::atoi(e));
  for (int t0 = 0; t0 < ntiles; t0 += chunk) {
    const int n = std::min(chunk, ntiles - t0), units = n * rounds;
    int* cnt = (int*)s->wf[R::WF_CNT];
    int* err = cnt + 15;  // the device's error word: bit 0 a parent out of range, bit 1 a dropped child
    HIPCHK(hipMemsetAsync(cnt, 0, 16 * sizeof(int), st));
    WfNode* node0 = (WfNode*)s->wf[R::WF_NODE0];
    double* scol = (double*)s->wf[R::WF_SCOL];
    uint8_t* straced = (uint8_t*)s->wf[R::WF_TRACED];
    hipLaunchKernelGGL(dv::wf_camera_kernel<F>, dim3(units), dim3(64), dv::LDS_RENDER_BYTES, st, sd, P, t0, rounds, node0,
                       scol, straced, (WfRay*)s->wf[R::WF_Q1], cnt + 1, (int32_t)(2 * (size_t)units * 64 / qdiv), err);
    HIPCHK(hipGetLastError());
    int counts[9] = {0};
    int L = 1;
    int cap = (int)(2 * (size_t)units * 64 / qdiv);  // the capacity the producing launch wrote its queue with
    for (; L <= 7; ++L) {  // level L reads queue L % 2 (WF_Q0 / WF_Q1), writes the other one
      int c = 0, bad = 0;
      HIPCHK(hipMemcpyAsync(&c, cnt + L, sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&bad, err, sizeof(int), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (bad || c > cap)  // the device dropped a ray or a delivery: stop before anything reads the queue
        return set_error(RT_E_HIP, std::string("RT_RENDER_WAVEFRONT: the device dropped ") +
                                       ((bad & 1) ? "a delivery (parent out of range)" : "a queued ray (queue capacity)"));
      if (c == 0) break;
      counts[L] = c;
      cap = 2 * c / qdiv;
      const int qin = (L % 2) ? R::WF_Q1 : R::WF_Q0, qout = (L % 2) ? R::WF_Q0 : R::WF_Q1;
      if ((rc = wf_grow(s, R::WF_NODE1 + L - 1, (size_t)c * sizeof(WfNode))) ||
          (rc = wf_grow(s, qout, (size_t)2 * c * sizeof(WfRay))))
        return rc;
      WfNode* prev = L == 1 ? node0 : (WfNode*)s->wf[R::WF_NODE1 + L - 2];
      const int32_t nPrev = L == 1 ? units * 64 : counts[L - 1];
      hipLaunchKernelGGL(dv::wf_level_kernel<F>, dim3((unsigned)((c + 63) / 64)), dim3(64), dv::LDS_RENDER_BYTES, st, sd, P,
                         (const WfRay*)s->wf[qin], cnt + L, (WfNode*)s->wf[R::WF_NODE1 + L - 1], prev, nPrev,
                         (WfRay*)s->wf[qout], cnt + L + 1, cap, err);
      HIPCHK(hipGetLastError());
    }
    for (int l = L - 1; l >= 1; --l) {  // bottom up: a level's frames into their parents
      WfNode* prev = l == 1 ? node0 : (WfNode*)s->wf[R::WF_NODE1 + l - 2];
      const int32_t nPrev = l == 1 ? units * 64 : counts[l - 1];
      hipLaunchKernelGGL(dv::wf_fold_kernel<F>, dim3((unsigned)((counts[l] + 255) / 256)), dim3(256), 0, st, sd,
                         (const WfNode*)s->wf[R::WF_NODE1 + l - 1], cnt + l, 0, prev, nPrev, scol, err);
    }
    hipLaunchKernelGGL(dv::wf_fold_kernel<F>, dim3((unsigned)((units * 64 + 255) / 256)), dim3(256), 0, st, sd,
                       (const WfNode*)node0, (const int*)nullptr, units * 64, (WfNode*)nullptr, 0, scol, err);
    hipLaunchKernelGGL(dv::wf_final_kernel<F>, dim3(n), dim3(64), 0, st, P, t0, rounds, (const double*)scol,
                       (const uint8_t*)straced, d_rgb, d_argb, dof);
    HIPCHK(hipGetLastError());
    int bad = 0;
    HIPCHK(hipMemcpyAsync(&bad, err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (bad)
      return set_error(RT_E_HIP, std::string("RT_RENDER_WAVEFRONT: the device dropped a ") +
                                     ((bad & 2) ? "queued ray (queue capacity)" : "delivery (parent out of range)"));
  }
  return RT_OK;
}
static int render_wavefront(rt_scene* s, const SceneD& sd, const ParamsD& P, uint32_t flags, float* d_rgb, int32_t* d_argb,
                            hipStream_t st) {
  const uint32_t f = (flags & RT_RENDER_GENERIC) ? (uint32_t)dv::FT_ALL : scene_features(s->hs);
  constexpr uint32_t C4 = dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX;
  if (f == 0) return render_wf<0u>(s, sd, P, d_rgb, d_argb, st);
  if ((f & ~C4) == 0) return render_wf<C4>(s, sd, P, d_rgb, d_argb, st);
  return render_wf<dv::FT_ALL>(s, sd, P, d_rgb, d_argb, st);
}

// the scene view a launch uses: nearest-first / wave-cull bits, or the reference's full scan
static SceneD launch_scene(const rt_scene* s, uint32_t flags) {
  SceneD sd = s->dev;
  sd.fastSlab |= SCENE_NEAREST_FIRST;
  if (sd.ntop <= 64 && !(flags & RT_RENDER_NOWAVECULL)) sd.fastSlab |= SCENE_WAVE_CULL;
  if (flags & RT_RENDER_NOCULL) { sd.topBound = s->noCullBound; sd.fastSlab &= ~(SCENE_NEAREST_FIRST | SCENE_WAVE_CULL); }
  return sd;
}

// tiles: an explicit tile list (rt_render_tiles_device) -- ntiles blocks, block b renders tiles[b]
static int launch(rt_scene* s, const ParamsD& P0, uint32_t flags, float* d_rgb, int32_t* d_argb, bool count,
                  hipStream_t st, const int32_t* tiles = nullptr, int ntiles = 0) {
  ParamsD P = P0;
  int tilesX = ((P.W + P.colStep - 1) / P.colStep + P.tw - 1) / P.tw, tilesY = (P.nrows + P.th - 1) / P.th;
  dim3 grid(dv::xcd_grid(tilesX * tilesY)), block(64);
  if ((flags & RT_RENDER_WAVEFRONT) && !count) {
    if (tiles) return set_error(RT_E_INVALID, "RT_RENDER_WAVEFRONT renders whole layouts, not tile lists");
    const SceneD sd = launch_scene(s, flags);
    if (P.colStep != 1) return set_error(RT_E_INVALID, "RT_RENDER_WAVEFRONT: not for refine passes");
    return render_wavefront(s, sd, P, flags, d_rgb, d_argb, st);
  }
  if (tiles) {
    P.order = const_cast<int32_t*>(tiles);
    P.tcost = nullptr;
    grid = dim3(ntiles);
  }
#ifndef RT_NO_SCHEDULE
  else if (!(flags & RT_RENDER_ROWMAJOR)) {
    int rc = schedule(s, P, count, st);
    if (rc) return rc;
  }
#endif
  const SceneD sd = launch_scene(s, flags);
  if (count) {  // the counting instantiation of the timed variant (count_variant)
    HIPCHK(hipMemsetAsync(s->counters, 0, sizeof(unsigned long long) * RT_ST_N, st));
    hipLaunchKernelGGL(count_variant(s->hs, flags).fn, grid, block, dv::LDS_RENDER_BYTES, st, sd, P, d_rgb, d_argb,
                       (unsigned long long*)s->counters);
  } else {
    hipLaunchKernelGGL(pick_variant(s->hs, flags), grid, block, dv::LDS_RENDER_BYTES, st, sd, P, d_rgb, d_argb,
                       (unsigned long long*)nullptr);
  }
  HIPCHK(hipGetLastError());
  if (P.tcost) {  // a measuring launch: mark its completion for sort_tiles
    for (auto& e : s->schedules)
      if (e.cost == P.tcost) {
        if (!e.measured) {
          hipEvent_t ev;
          HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
          e.measured = ev;
        }
        HIPCHK(hipEventRecord((hipEvent_t)e.measured, st));
      }
  }
  return RT_OK;
}

static int render_host(rt_scene* s, const rt_render_params* p, float* rgb, int32_t* argb, uint64_t* stats) {
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  HIPCHK(hipSetDevice(s->device));
  if (!s->stream) {
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    s->stream = st;
  }
  hipStream_t st = (hipStream_t)s->stream;
  const size_t npx = (size_t)P.nrows * P.W;
  if (npx > s->outCap) {  // grow-only device output buffers, reused by later calls
    HIPCHK(hipStreamSynchronize(st));
    (void)hipFree(s->outRgb);
    (void)hipFree(s->outArgb);
    s->outRgb = nullptr; s->outArgb = nullptr; s->outCap = 0;
    HIPCHK(hipMalloc(&s->outRgb, npx * 3 * sizeof(float)));
    HIPCHK(hipMalloc(&s->outArgb, npx * sizeof(int32_t)));
    s->outCap = npx;
  }
  // the read-back goes through pinned staging (a DMA at link speed; a copy into pageable memory is
  // staged by the runtime in small pieces), then one host memcpy into the caller's buffers
  const size_t nb = (rgb ? npx * 3 * sizeof(float) : 0) + (argb ? npx * sizeof(int32_t) : 0);
  if (nb > s->stageCap) {
    HIPCHK(hipStreamSynchronize(st));
    (void)hipHostFree(s->stage);
    s->stage = nullptr; s->stageCap = 0;
    HIPCHK(hipHostMalloc(&s->stage, nb, hipHostMallocDefault));
    s->stageCap = nb;
  }
  char* stg = (char*)s->stage;
  const size_t nrgb = rgb ? npx * 3 * sizeof(float) : 0;
  rc = launch(s, P, p->flags, s->outRgb, s->outArgb, stats != nullptr, st);
  hipError_t e = hipSuccess;
  if (rc == RT_OK && rgb) e = hipMemcpyAsync(stg, s->outRgb, nrgb, hipMemcpyDeviceToHost, st);
  if (rc == RT_OK && e == hipSuccess && argb) e = hipMemcpyAsync(stg + nrgb, s->outArgb, npx * sizeof(int32_t), hipMemcpyDeviceToHost, st);
  if (rc == RT_OK && e == hipSuccess && stats)
    e = hipMemcpyAsync(stats, s->counters, sizeof(uint64_t) * RT_ST_N, hipMemcpyDeviceToHost, st);
  hipError_t se = hipStreamSynchronize(st);  // the call blocks until the frame is in the caller's buffers
  if (rc == RT_OK && e != hipSuccess) rc = set_error(RT_E_HIP, hipGetErrorString(e));
  if (rc == RT_OK && se != hipSuccess) rc = set_error(RT_E_HIP, std::string("render kernel: ") + hipGetErrorString(se));
  if (rc == RT_OK && rgb) std::memcpy(rgb, stg, nrgb);
  if (rc == RT_OK && argb) std::memcpy(argb, stg + nrgb, npx * sizeof(int32_t));
  return rc;
}

// fdlibm sin / cos / asin / acos (csrc/jfdlibm.h) evaluated on the device: the parity
// self-check that device and host (oracle) results are bit-identical
__global__ void math_eval_kernel(const double* __restrict__ x, double* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  out[4 * i + 0] = jf::sin(v);
  out[4 * i + 1] = jf::cos(v);
  out[4 * i + 2] = jf::asin(v);
  out[4 * i + 3] = jf::acos(v);
}

extern "C" {

int rt_render(rt_scene* s, const rt_render_params* p, float* rgb, int32_t* argb) { return render_host(s, p, rgb, argb, nullptr); }

int rt_math_eval(const double* x, double* out, int64_t n, int device) {
  if (n < 0 || (n > 0 && (!x || !out))) return set_error(RT_E_INVALID, "rt_math_eval: bad arguments");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return set_error(RT_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= nd) return set_error(RT_E_INVALID, "device ordinal out of range");
  if (n == 0) return RT_OK;
  HIPCHK(hipSetDevice(device));
  double *dx = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(&dx, sizeof(double) * n));
  hipError_t e = hipMalloc(&dout, sizeof(double) * 4 * n);
  if (e == hipSuccess) e = hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(math_eval_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dout);
  if (e != hipSuccess) return set_error(RT_E_HIP, hipGetErrorString(e));
  return RT_OK;
}

int rt_photon_gather(rt_scene* s, const double* pts, double* out, int64_t n) {
  if (!s || n < 0 || (n > 0 && (!pts || !out))) return set_error(RT_E_INVALID, "rt_photon_gather: bad arguments");
  if (!s->photonsUploaded) return set_error(RT_E_INVALID, "rt_photon_gather: no photon map (rt_photons_build / rt_photons_set)");
  if (n == 0) return RT_OK;
  HIPCHK(hipSetDevice(s->device));
  double *dp = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(&dp, sizeof(double) * 3 * n));
  hipError_t e = hipMalloc(&dout, sizeof(double) * 3 * n);
  if (e == hipSuccess) e = hipMemcpy(dp, pts, sizeof(double) * 3 * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(dv::gather_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), dv::LDS_RENDER_BYTES, 0, s->dev, dp,
                       dout, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(double) * 3 * n, hipMemcpyDeviceToHost);
  (void)hipFree(dp);
  (void)hipFree(dout);
  if (e != hipSuccess) return set_error(RT_E_HIP, hipGetErrorString(e));
  return RT_OK;
}

int rt_render_variant(const rt_scene* s, uint32_t flags, uint32_t* timed, uint32_t* counted) {
  if (!s) return set_error(RT_E_INVALID, "rt_render_variant: null scene");
  if (timed) *timed = variant_mask(s->hs, flags);
  if (counted) *counted = count_variant(s->hs, flags).mask;
  return RT_OK;
}

int rt_render_count(rt_scene* s, const rt_render_params* p, float* rgb, int32_t* argb, uint64_t* stats) {
  if (!stats) return set_error(RT_E_INVALID, "null stats");
  return render_host(s, p, rgb, argb, stats);
}

int rt_render_device(rt_scene* s, const rt_render_params* p, float* d_rgb, int32_t* d_argb, void* stream) {
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  HIPCHK(hipSetDevice(s->device));
  return launch(s, P, p->flags, d_rgb, d_argb, false, (hipStream_t)stream);
}

static void tile_layout(const ParamsD& P, int32_t out[4]) {
  const int ncols = (P.W + P.colStep - 1) / P.colStep, tilesX = (ncols + P.tw - 1) / P.tw;
  out[0] = tilesX * ((P.nrows + P.th - 1) / P.th);
  out[1] = tilesX;
  out[2] = P.tw;
  out[3] = P.th;
}

int rt_tile_layout(rt_scene* s, const rt_render_params* p, int32_t* out) {
  if (!out) return set_error(RT_E_INVALID, "rt_tile_layout: null out");
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  tile_layout(P, out);
  return RT_OK;
}

int rt_tile_costs(rt_scene* s, const rt_render_params* p, uint32_t* cost, int cap) {
  if (!cost || cap < 0) return set_error(RT_E_INVALID, "rt_tile_costs: bad buffer");
  if (p && (p->flags & RT_RENDER_ROWMAJOR)) return set_error(RT_E_INVALID, "rt_tile_costs: RT_RENDER_ROWMAJOR has no costs");
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  int32_t lay[4];
  tile_layout(P, lay);
  if (P.nrows * (int64_t)((P.W + P.colStep - 1) / P.colStep) < (1 << 16)) {  // not scheduled: unit costs
    for (int i = 0; i < lay[0] && i < cap; ++i) cost[i] = 1;
    return lay[0];
  }
  // plain renders of the layout until one has measured its waves (schedule(): state >= 1)
  for (int it = 0; it < 3; ++it) {
    rt_scene::TileSchedule* e = nullptr;
    char key[160];
    std::snprintf(key, sizeof(key), "%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%.17g", P.W, P.H, P.row0, P.nrows, P.rowStep, P.band,
                  P.colStep, P.tw, P.th, P.G, P.viewZ);
    for (auto& x : s->schedules)
      if (x.key == key) { e = &x; break; }
    if (e && e->state >= 1) {
      HIPCHK(hipSetDevice(s->device));
      if (s->stream) HIPCHK(hipStreamSynchronize((hipStream_t)s->stream));
      if (e->measured) HIPCHK(hipEventSynchronize((hipEvent_t)e->measured));
      std::vector<uint32_t> c(e->ntiles);
      HIPCHK(hipMemcpy(c.data(), e->cost, sizeof(uint32_t) * e->ntiles, hipMemcpyDeviceToHost));
      for (int i = 0; i < e->ntiles && i < cap; ++i) cost[i] = c[i];
      return e->ntiles;
    }
    rt_render_params q = *p;
    q.flags &= ~(uint32_t)RT_RENDER_ROWMAJOR;
    rc = render_host(s, &q, nullptr, nullptr, nullptr);
    if (rc) return rc;
  }
  return set_error(RT_E_INVALID, "rt_tile_costs: the layout was not measured");
}

// the device copy of a validated tile list (rt_render_tiles_device / rt_render_tiles_count)
static int tile_list(rt_scene* s, const ParamsD& P, const int32_t* tiles, int ntiles, const int32_t** dev) {
  if (!tiles || ntiles <= 0) return set_error(RT_E_INVALID, "tile list: empty");
  if (dv::XCD_CHUNKS != 0) return set_error(RT_E_INVALID, "tile list: built with RT_XCD_CHUNKS");
  int32_t lay[4];
  tile_layout(P, lay);
  if (ntiles > lay[0]) return set_error(RT_E_INVALID, "tile list: more tiles than the layout has");
  rt_scene::TileList* L = nullptr;
  for (auto& x : s->tileLists)
    if (x.host.size() == (size_t)ntiles && std::memcmp(x.host.data(), tiles, sizeof(int32_t) * ntiles) == 0) { L = &x; break; }
  // a cached list (maybe validated as a pixel list, against another bound) is reused only below this layout's
  if (L && L->maxv >= lay[0]) return set_error(RT_E_INVALID, "tile list: tile index out of range");
  if (!L) {
    int32_t mx = -1;
    for (int i = 0; i < ntiles; ++i) {
      if (tiles[i] < 0 || tiles[i] >= lay[0]) return set_error(RT_E_INVALID, "tile list: tile index out of range");
      mx = std::max(mx, tiles[i]);
    }
    if (s->tileLists.size() >= 16) {  // oldest out (its launches may be on streams we do not know: drain the device)
      HIPCHK(hipDeviceSynchronize());
      (void)hipFree(s->tileLists.front().dev);
      s->tileLists.erase(s->tileLists.begin());
    }
    rt_scene::TileList t;
    t.host.assign(tiles, tiles + ntiles);
    t.maxv = mx;
    HIPCHK(hipMalloc(&t.dev, sizeof(int32_t) * ntiles));
    HIPCHK(hipMemcpy(t.dev, tiles, sizeof(int32_t) * ntiles, hipMemcpyHostToDevice));
    s->tileLists.push_back(std::move(t));
    L = &s->tileLists.back();
  }
  *dev = L->dev;
  return RT_OK;
}

int rt_render_tiles_count(rt_scene* s, const rt_render_params* p, const int32_t* tiles, int ntiles, uint64_t* stats) {
  if (!stats) return set_error(RT_E_INVALID, "null stats");
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  HIPCHK(hipSetDevice(s->device));
  const int32_t* dt = nullptr;
  rc = tile_list(s, P, tiles, ntiles, &dt);
  if (rc) return rc;
  if (!s->stream) {
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    s->stream = st;
  }
  hipStream_t st = (hipStream_t)s->stream;
  const size_t npx = (size_t)P.nrows * P.W;
  float* d_rgb = nullptr;
  int32_t* d_argb = nullptr;
  HIPCHK(hipMalloc(&d_rgb, npx * 3 * sizeof(float)));
  hipError_t e = hipMalloc(&d_argb, npx * sizeof(int32_t));
  if (e == hipSuccess) rc = launch(s, P, p->flags, d_rgb, d_argb, true, st, dt, ntiles);
  if (e == hipSuccess && rc == RT_OK) e = hipMemcpyAsync(stats, s->counters, sizeof(uint64_t) * RT_ST_N, hipMemcpyDeviceToHost, st);
  hipError_t se = hipStreamSynchronize(st);
  (void)hipFree(d_rgb);
  (void)hipFree(d_argb);
  if (rc == RT_OK && e != hipSuccess) rc = set_error(RT_E_HIP, hipGetErrorString(e));
  if (rc == RT_OK && se != hipSuccess) rc = set_error(RT_E_HIP, std::string("count kernel: ") + hipGetErrorString(se));
  return rc;
}

}  // extern "C"

template <uint32_t F>
static int launch_pixels(const SceneD& sd, const ParamsD& P, const int32_t* dpix, int npix, double* smpCol,
                         uint8_t* smpTr, float* d_rgb, int32_t* d_argb, hipStream_t st) {
  const int dof = ((F & dv::FT_DOF) && sd.dof && !((F & dv::FT_CAMX) && P.cam != 0)) ? 1 : 0;
  hipLaunchKernelGGL(dv::sample_kernel<F>, dim3((unsigned)((int64_t)npix * P.spp)), dim3(64), dv::LDS_RENDER_BYTES, st, sd,
                     P, dpix, smpCol, smpTr);
  hipLaunchKernelGGL(dv::pixel_sum_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, P, dpix, npix,
                     (const double*)smpCol, (const uint8_t*)smpTr, d_rgb, d_argb, dof);
  HIPCHK(hipGetLastError());
  return RT_OK;
}

// one sample per wave for a device pixel list (validated by the caller), per-sample colours in
// smpCol[npix * spp * 3] / smpTr[npix * spp]
static int pixel_samples(rt_scene* s, const ParamsD& P, uint32_t flags, const int32_t* dpix, int npix, double* smpCol,
                         uint8_t* smpTr, float* d_rgb, int32_t* d_argb, hipStream_t st) {
  const SceneD sd = launch_scene(s, flags);
  const uint32_t f = (flags & RT_RENDER_GENERIC) ? (uint32_t)dv::FT_ALL : scene_features(s->hs);
  constexpr uint32_t C4 = dv::FT_PRIM | dv::FT_TRANS | dv::FT_TEX | dv::FT_LIGHTX;
  if (f == 0) return launch_pixels<0u>(sd, P, dpix, npix, smpCol, smpTr, d_rgb, d_argb, st);
  if ((f & ~dv::F_C5) == 0) return launch_pixels<dv::F_C5>(sd, P, dpix, npix, smpCol, smpTr, d_rgb, d_argb, st);
  if ((f & ~C4) == 0) return launch_pixels<C4>(sd, P, dpix, npix, smpCol, smpTr, d_rgb, d_argb, st);
  return launch_pixels<dv::FT_ALL>(sd, P, dpix, npix, smpCol, smpTr, d_rgb, d_argb, st);
}

extern "C" {

int rt_render_pixels_device(rt_scene* s, const rt_render_params* p, const int32_t* pixels, int npix, float* d_rgb,
                            int32_t* d_argb, void* stream) {
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  if (P.row0 != 0 || P.nrows != P.H || P.rowStep != 1 || P.band != 1)
    return set_error(RT_E_INVALID, "rt_render_pixels_device: whole-frame layouts only");
  if (!pixels || npix <= 0) return set_error(RT_E_INVALID, "rt_render_pixels_device: empty pixel list");
  if ((int64_t)npix * P.spp > INT32_MAX) return set_error(RT_E_INVALID, "rt_render_pixels_device: too many samples");
  for (int i = 0; i < npix; ++i)
    if (pixels[i] < 0 || (int64_t)pixels[i] >= (int64_t)P.W * P.H) return set_error(RT_E_INVALID, "rt_render_pixels_device: pixel out of range");
  HIPCHK(hipSetDevice(s->device));
  // the list's device copy: the validated-list cache of the tile lists (a list of ints either way;
  // its range check there is against the tile count, so bound it by the pixel count here)
  const int32_t* dpix = nullptr;
  {
    rt_scene::TileList* L = nullptr;
    for (auto& x : s->tileLists)
      if (x.host.size() == (size_t)npix && std::memcmp(x.host.data(), pixels, sizeof(int32_t) * npix) == 0) { L = &x; break; }
    if (!L) {
      if (s->tileLists.size() >= 16) {
        HIPCHK(hipDeviceSynchronize());
        (void)hipFree(s->tileLists.front().dev);
        s->tileLists.erase(s->tileLists.begin());
      }
      rt_scene::TileList t;
      t.host.assign(pixels, pixels + npix);
      t.maxv = *std::max_element(pixels, pixels + npix);
      HIPCHK(hipMalloc(&t.dev, sizeof(int32_t) * npix));
      HIPCHK(hipMemcpy(t.dev, pixels, sizeof(int32_t) * npix, hipMemcpyHostToDevice));
      s->tileLists.push_back(std::move(t));
      L = &s->tileLists.back();
    }
    dpix = L->dev;
  }
  const size_t ns = (size_t)npix * P.spp;
  if (ns > s->smpCap) {  // grow-only; earlier launches may still read the old buffers: drain the device
    HIPCHK(hipDeviceSynchronize());
    (void)hipFree(s->smpCol);
    (void)hipFree(s->smpTr);
    s->smpCol = s->smpTr = nullptr;
    s->smpCap = 0;
    HIPCHK(hipMalloc(&s->smpCol, ns * 3 * sizeof(double)));
    HIPCHK(hipMalloc(&s->smpTr, ns));
    s->smpCap = ns;
  }
  return pixel_samples(s, P, p->flags, dpix, npix, (double*)s->smpCol, (uint8_t*)s->smpTr, d_rgb, d_argb,
                       (hipStream_t)stream);
}

int rt_render_tiles_device(rt_scene* s, const rt_render_params* p, const int32_t* tiles, int ntiles, float* d_rgb,
                           int32_t* d_argb, void* stream) {
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  HIPCHK(hipSetDevice(s->device));
  const int32_t* dt = nullptr;
  rc = tile_list(s, P, tiles, ntiles, &dt);
  if (rc) return rc;
  return launch(s, P, p->flags, d_rgb, d_argb, false, (hipStream_t)stream, dt, ntiles);
}

int rt_time_render(rt_scene* s, const rt_render_params* p, int warmup, int iters, double* avg_ms) {
  if (!avg_ms || iters <= 0) return set_error(RT_E_INVALID, "bad timing arguments");
  ParamsD P;
  int rc = make_params(s, p, P);
  if (rc) return rc;
  HIPCHK(hipSetDevice(s->device));
  size_t npx = (size_t)P.nrows * P.W;
  float* d_rgb = nullptr;
  int32_t* d_argb = nullptr;
  HIPCHK(hipMalloc(&d_rgb, npx * 3 * sizeof(float)));
  HIPCHK(hipMalloc(&d_argb, npx * sizeof(int32_t)));
  hipStream_t st;
  HIPCHK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  // >= 2 warmups: the tile schedule's measuring render and its re-sort stay out of the timed launches
  for (int i = 0; i < std::max(warmup, 2) && rc == RT_OK; ++i) rc = launch(s, P, p->flags, d_rgb, d_argb, false, st);
  if (rc == RT_OK) {
    HIPCHK(hipEventRecord(e0, st));
    for (int i = 0; i < iters && rc == RT_OK; ++i) rc = launch(s, P, p->flags, d_rgb, d_argb, false, st);
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / iters;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(st);
  (void)hipFree(d_rgb);
  (void)hipFree(d_argb);
  return rc;
}

// myScene.setRefine (myScene.java:796-803): refIDX = (int)(log10(.5 (W + H) / 16) / log10 2),
// steps pow2[refIDX], ..., pow2[0] (the image size is the render's, as for viewZ)
int rt_refine_steps(const rt_scene* s, int width, int height, int* steps, int cap) {
  if (!s || width <= 0 || height <= 0) return set_error(RT_E_INVALID, "rt_refine_steps: bad argument");
  int n = 1;
  int st[16] = {1};
  if (s->refine) {
    const int refIDX = (int)(std::log10(.5 * (width + height) / 16.0) / std::log10(2.0));
    if (refIDX >= 0) {
      n = std::min(refIDX, 15) + 1;
      for (int i = n - 1; i >= 0; --i) st[n - 1 - i] = 1 << i;
    }
  }
  for (int i = 0; i < n && i < cap && steps; ++i) steps[i] = st[i];
  return n;
}

// One `refine` pass of myFOVScene.draw (myScene.java:1481-1531; fisheye / ortho / DOF alike):
// the pixels (row, col) with row, col multiples of `step`, each written over its step x step
// span (writePxlSpan, :1171-1177) in full-size host buffers; skip_origin leaves (0,0) alone
// (`skipPxl`, every pass after the first). Pixel RNG keys are those of the full render, so
// the last pass (step 1) reproduces rt_render everywhere but a skipped (0,0).
int rt_render_pass(rt_scene* s, const rt_render_params* p, int step, int skip_origin, float* rgb, int32_t* argb) {
  if (!s || !p || step <= 0) return set_error(RT_E_INVALID, "rt_render_pass: bad argument");
  rt_render_params q = *p;
  q.row0 = 0; q.row1 = p->height; q.row_step = step; q.row_band = 1;
  ParamsD P;
  int rc = make_params(s, &q, P);
  if (rc) return rc;
  P.colStep = step;
  HIPCHK(hipSetDevice(s->device));
  const int W = P.W, H = P.H, ncols = (W + step - 1) / step, nr = P.nrows;
  const size_t npx = (size_t)nr * ncols;
  float* d_rgb = nullptr;
  int32_t* d_argb = nullptr;
  HIPCHK(hipMalloc(&d_rgb, npx * 3 * sizeof(float)));
  hipError_t e = hipMalloc(&d_argb, npx * sizeof(int32_t));
  if (e != hipSuccess) { (void)hipFree(d_rgb); return set_error(RT_E_HIP, hipGetErrorString(e)); }
  // a pass with step > 1 needs the column step (FT_PASS): the all-features kernel
  rc = launch(s, P, step > 1 ? (p->flags | RT_RENDER_GENERIC) : p->flags, d_rgb, d_argb, false, 0);
  std::vector<float> hr;
  std::vector<int32_t> ha;
  if (rc == RT_OK) {
    e = hipDeviceSynchronize();
    if (e == hipSuccess) { hr.resize(npx * 3); e = hipMemcpy(hr.data(), d_rgb, npx * 3 * sizeof(float), hipMemcpyDeviceToHost); }
    if (e == hipSuccess) { ha.resize(npx); e = hipMemcpy(ha.data(), d_argb, npx * sizeof(int32_t), hipMemcpyDeviceToHost); }
    if (e != hipSuccess) rc = set_error(RT_E_HIP, std::string("render pass: ") + hipGetErrorString(e));
  }
  (void)hipFree(d_rgb);
  (void)hipFree(d_argb);
  if (rc) return rc;
  for (int r = 0; r < nr; ++r)
    for (int c = 0; c < ncols; ++c) {
      const int row = r * step, col = c * step;
      if (skip_origin && row == 0 && col == 0) continue;
      const size_t i = (size_t)r * ncols + c;
      for (int y = row; y < std::min(row + step, H); ++y)
        for (int x = col; x < std::min(col + step, W); ++x) {
          const size_t o = (size_t)y * W + x;
          if (argb) argb[o] = ha[i];
          if (rgb) { rgb[3 * o] = hr[3 * i]; rgb[3 * o + 1] = hr[3 * i + 1]; rgb[3 * o + 2] = hr[3 * i + 2]; }
        }
    }
  return RT_OK;
}

#ifdef RT_PROF_PKSTAT
int rt_prof_pkstat_get(uint64_t* out) {  // profiling builds only: read and clear rt_pk_stat[16]
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(dv::rt_pk_stat), 16 * sizeof(uint64_t)));
  const uint64_t z[16] = {};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dv::rt_pk_stat), z, sizeof(z)));
  return RT_OK;
}
#endif
#ifdef RT_PROF_REGIONS
int rt_prof_regions_get(uint64_t* out) {  // profiling builds only: read and clear rt_prof_reg[16]
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(dv::rt_prof_reg), dv::R_N * sizeof(uint64_t)));
  const uint64_t z[dv::R_N] = {};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dv::rt_prof_reg), z, sizeof(z)));
  return RT_OK;
}
#endif
#ifdef RT_PROF_TIMELINE
int rt_prof_timeline_set(void* d_buf) {  // profiling builds only
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(dv::rt_tl_buf), &d_buf, sizeof(void*)));
  return RT_OK;
}
#endif

}  // extern "C"

int rt_upload_photons(rt_scene* s);

// Shoot photons [first, first+count) of every light (myScene.sendCausticPhotons :952-998 /
// sendDiffusePhotons :1000-1091 with the emitted-photon index range restricted) into
// pos/pwr in photon_list order: light, photon index, path slot. Chunked so the
// per-lane slot buffers stay bounded for any photon count.
int rt::shoot_photons(rt_scene* s, uint64_t seed, int64_t first, int64_t count, std::vector<double>& pos,
                      std::vector<double>& pwr, std::vector<int64_t>& perLight) {
  HostScene& h = s->hs;
  pos.clear();
  pwr.clear();
  perLight.assign(h.light.size(), 0);
  const long total = (long)h.light.size() * count;
  if (total <= 0) return RT_OK;
  HIPCHK(hipSetDevice(s->device));
  const long CH = std::min<long>(total, 1L << 22);
  dv::PhotonOut* d_out = nullptr;
  int* d_cnt = nullptr;
  HIPCHK(hipMalloc(&d_out, sizeof(dv::PhotonOut) * dv::PH_SLOTS * CH));
  hipError_t e = hipMalloc(&d_cnt, sizeof(int) * CH);
  const bool caustic = h.photonMode == 2;
  const double pwrMult = (caustic ? 40.0 : 8.0) / h.photonCount;  // causticsLightPwrMult / diffuseLightPwrMult (myScene.java:109-110)
  std::vector<int> cnt(CH);
  std::vector<dv::PhotonOut> out((size_t)dv::PH_SLOTS * CH);
  for (long base = 0; base < total && e == hipSuccess; base += CH) {
    const long n = std::min(CH, total - base);
    if (scene_features(h) & dv::FT_INST)
      hipLaunchKernelGGL(dv::photon_kernel<dv::FT_ALL>, dim3((unsigned)((n + 63) / 64)), dim3(64), dv::LDS_BYTES, 0,
                         s->dev, seed, (long)first, (long)count, base, n, caustic ? 1 : 0, pwrMult, d_out, d_cnt);
    else
      hipLaunchKernelGGL(dv::photon_kernel<dv::FT_ALL & ~dv::FT_INST>, dim3((unsigned)((n + 63) / 64)), dim3(64),
                         dv::LDS_BYTES, 0, s->dev, seed, (long)first, (long)count, base, n, caustic ? 1 : 0, pwrMult,
                         d_out, d_cnt);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(cnt.data(), d_cnt, sizeof(int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out.data(), d_out, sizeof(dv::PhotonOut) * dv::PH_SLOTS * n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) break;
    for (long g = 0; g < n; ++g)
      for (int j = 0; j < cnt[g]; ++j) {
        const dv::PhotonOut& p = out[(size_t)g * dv::PH_SLOTS + j];
        pos.insert(pos.end(), p.pos, p.pos + 3);
        pwr.insert(pwr.end(), p.pwr, p.pwr + 3);
        perLight[(base + g) / count]++;
      }
  }
  (void)hipFree(d_out);
  (void)hipFree(d_cnt);
  if (e != hipSuccess) return set_error(RT_E_HIP, std::string("photon pre-pass: ") + hipGetErrorString(e));
  return RT_OK;
}

int rt::check_photon_params(const HostScene& h) {
  if (h.photonMode == 0) return set_error(RT_E_INVALID, "scene has no photon map");
  if (h.photonCount <= 0 || h.photonK <= 0) return set_error(RT_E_INVALID, "bad photon parameters");
  if (h.photonK > dv::KNN_MAX) return set_error(RT_E_INVALID, "photon neighbourhood k > 256 unsupported");
  return RT_OK;
}

// The photon map of photon_list: built on the device (photon_build.hip) unless it fits one
// leaf or DISTRAYTRACER_PHOTON_BUILD=host asks for the host build (csrc/photon.cpp; the two
// are identical -- a GPU test checks it).
int rt::set_photon_map(rt_scene* s, std::vector<double>& pos, std::vector<double>& pwr) {
  HostScene& h = s->hs;
  const int64_t n = (int64_t)(pos.size() / 3);
  const char* mode = std::getenv("DISTRAYTRACER_PHOTON_BUILD");
  if (n > PHOTON_LEAF && !(mode && std::string(mode) == "host")) {
    HIPCHK(hipSetDevice(s->device));
    int rc = build_photon_tree_gpu(s, pos.data(), pwr.data(), n);
    h.photonListPos.swap(pos);
    h.photonListPwr.swap(pwr);
    return rc;
  }
  build_photon_tree(h, pos, pwr);
  return rt_upload_photons(s);
}

extern "C" int rt_photons_build(rt_scene* s, uint64_t seed) {
  if (!s) return set_error(RT_E_INVALID, "null scene");
  HostScene& h = s->hs;
  if (h.photonMode == 0 || s->photonsUploaded) return RT_OK;
  int rc = check_photon_params(h);
  if (rc) return rc;
  std::vector<double> pos, pwr;
  std::vector<int64_t> perLight;
  if ((rc = shoot_photons(s, seed, 0, h.photonCount, pos, pwr, perLight))) return rc;
  return set_photon_map(s, pos, pwr);
}

extern "C" int rt_photons_shoot(rt_scene* s, uint64_t seed, int64_t first, int64_t count, int64_t* per_light) {
  if (!s) return set_error(RT_E_INVALID, "null scene");
  HostScene& h = s->hs;
  int rc = check_photon_params(h);
  if (rc) return rc;
  if (first < 0 || count < 0 || first + count > h.photonCount) return set_error(RT_E_INVALID, "photon range out of bounds");
  std::vector<double> pos, pwr;
  std::vector<int64_t> perLight;
  if ((rc = shoot_photons(s, seed, first, count, pos, pwr, perLight))) return rc;
  h.photonListPos.swap(pos);
  h.photonListPwr.swap(pwr);
  h.nphoton = (int64_t)(h.photonListPos.size() / 3);
  if (per_light)
    for (size_t l = 0; l < perLight.size(); ++l) per_light[l] = perLight[l];
  return RT_OK;
}

extern "C" int rt_photons_set(rt_scene* s, const double* pos, const double* pwr, int64_t n) {
  if (!s || n < 0 || (n > 0 && (!pos || !pwr))) return set_error(RT_E_INVALID, "bad photon list");
  HostScene& h = s->hs;
  int rc = check_photon_params(h);
  if (rc) return rc;
  if (n > INT32_MAX / 4) return set_error(RT_E_INVALID, "photon map too large");
  std::vector<double> p(pos, pos + 3 * n), w(pwr, pwr + 3 * n);
  s->photonsUploaded = false;
  return set_photon_map(s, p, w);
}

extern "C" int rt_scene_photon_kdtree(const rt_scene* s, int32_t* out, int64_t n) {
  if (!s || n < 0 || (n > 0 && !out)) return set_error(RT_E_INVALID, "rt_scene_photon_kdtree: bad arguments");
  if (!s->photonsUploaded) return set_error(RT_E_INVALID, "rt_scene_photon_kdtree: no photon map");
  n = std::min<int64_t>(n, s->hs.nphoton);
  if (n == 0) return RT_OK;
  HIPCHK(hipSetDevice(s->device));
  int32_t off = 0;
  HIPCHK(hipMemcpy(&off, &s->dev.pnode[s->dev.photonRoot].padR[2], sizeof(int32_t), hipMemcpyDeviceToHost));
  if (off <= 0) return set_error(RT_E_INVALID, "rt_scene_photon_kdtree: the photon map has no kd-tree");
  HIPCHK(hipMemcpy(out, reinterpret_cast<const KdNodeD*>(s->dev.pnode + off), sizeof(KdNodeD) * n, hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_scene_photon_map(const rt_scene* s, void* nodes, int64_t node_cap, double* ppos, double* ppwr,
                                   int64_t n, int64_t* n_nodes, int32_t* root) {
  if (!s || !n_nodes) return set_error(RT_E_INVALID, "null argument");
  const HostScene& h = s->hs;
  *n_nodes = h.pnodeCount;
  if (root) *root = s->dev.photonRoot;
  if (!s->photonsUploaded) return RT_OK;
  HIPCHK(hipSetDevice(s->device));
  const int64_t nn = std::min<int64_t>(node_cap, h.pnodeCount), np = std::min<int64_t>(n, h.nphoton);
  if (nodes && nn > 0) HIPCHK(hipMemcpy(nodes, s->dev.pnode, sizeof(NodeD) * nn, hipMemcpyDeviceToHost));
  if (ppos && np > 0) HIPCHK(hipMemcpy(ppos, s->dev.ppos, sizeof(double) * 3 * np, hipMemcpyDeviceToHost));
  if (ppwr && np > 0) HIPCHK(hipMemcpy(ppwr, s->dev.ppwr, sizeof(double) * 3 * np, hipMemcpyDeviceToHost));
  return RT_OK;
}

// ---------------------------------------------------------------------------------------------
// internal entry points of the multi-GPU group (group.hip, rt_internal.h)
int rt::prepare_render(rt_scene* s, const rt_render_params* p, ParamsD& P) { return make_params(s, p, P); }

int rt::launch_tile_list(rt_scene* s, const ParamsD& P, uint32_t flags, const int32_t* dtiles, int ntiles, float* rgb,
                         int32_t* argb, void* stream) {
  if (ntiles <= 0) return RT_OK;
  return launch(s, P, flags & ~(uint32_t)RT_RENDER_WAVEFRONT, rgb, argb, false, (hipStream_t)stream, dtiles, ntiles);
}

int rt::launch_pixel_list(rt_scene* s, const ParamsD& P, uint32_t flags, const int32_t* dpix, int npix, double* smpCol,
                          uint8_t* smpTr, float* rgb, int32_t* argb, void* stream) {
  if (npix <= 0) return RT_OK;
  return pixel_samples(s, P, flags, dpix, npix, smpCol, smpTr, rgb, argb, (hipStream_t)stream);
}
