// ORACLE / TEST INFRASTRUCTURE ONLY.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library, and only as the checker. The product (distraytracer_old_amd/)
// never links or calls it.
//
// CPU restatement, in IEEE double, of the per-pixel / per-sample trace loop of
// jturner65/distRayTracer_old (Java 8 + Processing). The object model mirrors the
// reference class by class so that the recursion structure, tie-breaking and
// quirks are reproduced; every function cites the Java
// file:line it follows (paths relative to src/rayTracerDistAccelShdPhtnMap/).
//
// Parity status: the Java reference cannot be compiled or run here (no JDK), so
// the restatement is pinned by the hand-derived known-answer pixels of
// SURVEY.md 8(c) / BASELINE.md 6 (tests/test_oracle.py) and by committed golden
// fixtures it generates (tests/golden/). ThreadLocalRandom is replaced by the
// keyed counter RNG of jmath.h (the reference is not seedable).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <queue>
#include <sstream>
#include <string>
#include <vector>

#include "jmath.h"
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

struct Scene;
struct GeomBase;

// ---------------------------------------------------------------------------
// colours: myColor clamps every channel to <= 1 at construction (myObjShader.java:659-674)
struct Color {
  double r = 0, g = 0, b = 0;
  Color() {}
  Color(double _r, double _g, double _b) : r(jmin(1, _r)), g(jmin(1, _g)), b(jmin(1, _b)) {}
};
static inline Color color_from_int(uint32_t c) {  // myObjShader.java:663
  return Color(((c >> 16) & 0xFF) / 255.0, ((c >> 8) & 0xFF) / 255.0, (c & 0xFF) / 255.0);
}
static inline int32_t color_argb(const Color& c) {  // myObjShader.java:671 (+ not |, truncation)
  uint32_t v = (uint32_t)(255 << 24) + ((uint32_t)jd2i(c.r * 255) << 16) + ((uint32_t)jd2i(c.g * 255) << 8) +
               (uint32_t)jd2i(c.b * 255);
  return (int32_t)v;
}

struct Texture {  // decoded RGB8 image, Processing pixel ints
  int w = 0, h = 0;
  std::vector<uint32_t> px;
};

// ---------------------------------------------------------------------------
// ray (myRay.java:7-127) with the RNG key that replaces ThreadLocalRandom
struct RKey {
  uint64_t seed = 0, pixel = 0;
  uint32_t sample = 0, node = 0;
  uint32_t time_site = SITE_TIME;
  uint32_t time_k = 0;
};
struct Ray {
  V3 origin, direction;
  int gen = 0;
  double kt[5] = {1, 1, 1, 1, 1};  // currKTrans
  RKey key;
  double time = -1;
  Ray() {}
  Ray(const V3& o, const V3& d, int g) : origin(o), direction(d), gen(g) { normalize_ip(direction); }
  double get_time() {  // myRay.java:49-52, keyed
    if (time == -1) time = rng_range(rng_bits(key.seed, key.pixel, key.sample, key.node, key.time_site, key.time_k), 0, 1.0);
    return time;
  }
  V3 point(double t) const { return V3(direction.x * t + origin.x, direction.y * t + origin.y, direction.z * t + origin.z); }
};
// myRay.getTransformedRay (myRay.java:91-102): re-normalises the SOURCE ray's
// direction in place, then applies trans to (o,1) and (d,0) without renormalising.
static inline Ray transformed(Ray& ray, const M4& trans, uint32_t objkey) {
  normalize_ip(ray.direction);
  Ray r;
  r.origin = xpt(trans, ray.origin);
  r.direction = xvec(trans, ray.direction);
  r.gen = ray.gen;
  for (int i = 0; i < 5; ++i) r.kt[i] = ray.kt[i];
  r.key = ray.key;
  r.key.time_k = objkey;
  r.time = -1;
  return r;
}

struct Shader;
struct Hit {  // rayHit (myRay.java:130-186)
  bool isHit = false;
  double t = DMAX;
  GeomBase* obj = nullptr;
  Shader* shdr = nullptr;
  Ray transRay;
  V3 objNorm, hitLoc, fwdTransHitLoc, fwdTransRayDir;
  const CTM* ctm = nullptr;
  std::shared_ptr<CTM> ctm_own;  // reCalcCTMHitNorm's rebuilt array
  int args[2] = {0, 0};
  double ltMult = 1;
  double phtnPwr[3] = {0, 0, 0};
};

// stats shared with the product's counters (layout in DESIGN.md "Counters")
enum { ST_CAM = 0, ST_SHADOW, ST_REFL, ST_REFR, ST_BOX, ST_TRI, ST_QUAD, ST_SPHERE, ST_LIGHT, ST_PHOTON, ST_TEXEL, ST_N = 16 };

// ---------------------------------------------------------------------------
// geometry base (myGeomBase.java:10-87)
struct GeomBase {
  Scene* scene = nullptr;
  std::shared_ptr<CTM> ctm;
  V3 origin;
  V3 trans_origin;
  Shader* shdr = nullptr;
  V3 minVals{100000, 100000, 100000}, maxVals{-100000, -100000, -100000};
  struct BBox* bbox = nullptr;
  uint32_t key = 0;  // prim creation index (RNG key for per-object ray time)
  bool isLight = false;
  virtual ~GeomBase() {}
  virtual V3 getOrigin(double) { return origin; }
  virtual V3 getMaxVec() { return maxVals; }
  virtual V3 getMinVec() { return minVals; }
  virtual int shadowHit(Ray& ray, Ray& trans, const CTM* ctara, double distToLight, uint64_t* st);
  virtual Hit intersect(Ray& ray, Ray& trans, const CTM* ctara, uint64_t* st) = 0;
  virtual V3 normalAt(const V3& pt, const int* args) = 0;
  virtual void txtrCoords(const V3& pt, const int* args, const Texture& tex, double time, double& u, double& v) { u = v = 0; }
  virtual bool isAccel() const { return false; }
};

// objHit (myRay.java:119-125) + rayHit ctor (myRay.java:147-161)
static Hit obj_hit(Ray& transRay, GeomBase* obj, const V3& rawRayDir, const CTM* ct, const V3& pt, const int* args, double t) {
  Hit h;
  V3 n = xvec(ct->adj, obj->normalAt(pt, args));
  normalize_ip(n);
  h.transRay = transRay;
  h.isHit = true;
  h.obj = obj;
  h.shdr = obj->shdr;
  h.ctm = ct;
  h.objNorm = n;
  h.t = t;
  h.hitLoc = pt;
  h.fwdTransHitLoc = xpt(ct->g, pt);
  h.fwdTransRayDir = rawRayDir;
  if (args) { h.args[0] = args[0]; h.args[1] = args[1]; }
  h.ltMult = 1;
  return h;
}

// myBBox (myGeomBase.java:90-197)
struct BBox : GeomBase {
  GeomBase* owner = nullptr;
  BBox(Scene* s, const V3& mn, const V3& mx);
  void calc_min_max(const V3& mn, const V3& mx) {
    minVals = V3(jmin(mn.x, minVals.x), jmin(mn.y, minVals.y), jmin(mn.z, minVals.z));
    maxVals = V3(jmax(mx.x, maxVals.x), jmax(mx.y, maxVals.y), jmax(mx.z, maxVals.z));
  }
  void add_obj(GeomBase* o) { owner = o; ctm = o->ctm; }
  // slab test :132-162 -> returns hit flag, entry t and plane idx
  bool slab(const Ray& tr, double& tEntry, int& idx) const {
    double ro[3] = {tr.origin.x, tr.origin.y, tr.origin.z}, rd[3] = {tr.direction.x, tr.direction.y, tr.direction.z};
    double mn[3] = {minVals.x, minVals.y, minVals.z}, mx[3] = {maxVals.x, maxVals.y, maxVals.z};
    double t1[3], t2[3], tMin[3] = {DMAX, DMAX, DMAX}, tMax[3] = {-DMAX, -DMAX, -DMAX};
    double biggestMin = -DMAX;
    idx = -1;
    for (int i = 0; i < 3; ++i) {
      t1[i] = (mn[i] - ro[i]) / rd[i];
      t2[i] = (mx[i] - ro[i]) / rd[i];
    }
    for (int i = 0; i < 3; ++i) {
      if (t1[i] < t2[i]) {
        tMin[i] = t1[i]; tMax[i] = t2[i];
        if (biggestMin < t1[i]) { idx = i; biggestMin = t1[i]; }
      } else {
        tMin[i] = t2[i]; tMax[i] = t1[i];
        if (biggestMin < t2[i]) { idx = i + 3; biggestMin = t2[i]; }
      }
    }
    // p.min / p.max skip NaN (DistRayTracer.java:424-425)
    double mnv = DMAX, mxv = -DMAX;
    for (int i = 0; i < 3; ++i) { if (tMax[i] < mnv) mnv = tMax[i]; if (tMin[i] > mxv) mxv = tMin[i]; }
    tEntry = biggestMin;
    return (mnv > mxv) && biggestMin > 0;
  }
  // record-free slab hit used by accel traversal (box records never escape it)
  Hit slab_hit(const Ray& tr, uint64_t* st) const {
    if (st) st[ST_BOX]++;
    Hit h;
    double te;
    int idx;
    if (slab(tr, te, idx)) { h.isHit = true; h.t = te; }
    return h;
  }
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {
    if (st) st[ST_BOX]++;
    double te;
    int idx;
    if (!slab(tr, te, idx)) return Hit();
    int args[2] = {0, idx};
    V3 raw = xvec(ctara->g, tr.direction);
    return obj_hit(tr, owner, raw, ctara, tr.point(te), args, te);
  }
  int shadowHit(Ray& ray, Ray& tr, const CTM* ctara, double d, uint64_t* st) override {
    if (st) st[ST_BOX]++;
    double te;
    int idx;
    if (slab(tr, te, idx) && (d - te) > EPS) return 1;
    return 0;
  }
  V3 normalAt(const V3&, const int* args) override {
    switch (args[1]) {
      case 0: return V3(-1, 0, 0);
      case 1: return V3(0, -1, 0);
      case 2: return V3(0, 0, -1);
      case 3: return V3(1, 0, 0);
      case 4: return V3(0, 1, 0);
      case 5: return V3(0, 0, 1);
      default: return V3(0, 0, -1);
    }
  }
};

// ---------------------------------------------------------------------------
// shaders (myObjShader.java)
enum TexKind { TX_NONE = 0, TX_IMAGE = 1, TX_NOISE = 2, TX_WOOD = 3, TX_MARBLE = 4, TX_STONE = 5, TX_WOOD2 = 6 };
struct Shader {
  bool simple = false;  // mySimpleReflObjShdr
  Color diffuse, ambient, specular, curPermClr, KReflClr;
  V3 phtnDiffScl, phtnSpecScl, phtnPermClr;
  double avgDiffClr = 0, avgSpecClr = 0, avgPermClr = 0;
  double phongExp = 0, KRefl = 0, KTrans = 0, currPerm = 0, diffConst = 1;
  bool hasCaustic = false, usePhotonMap = false, isCausticPhtn = false;
  // texture handler
  int tex = TX_NONE;
  bool txTop = false;
  const Texture* texTop = nullptr;
  double scale = 1;  // noise textures
  int numOctaves = 8;
  double turbMult = 1, colorScale = 10, colorMult = .2;
  V3 periodMult{10, 10, 10};
  bool rndColors = false, useFwdTrans = false;
  std::vector<Color> colors;
  // myCellularTexture (myTextureHandler.java:380-498)
  int numPtsDist = 2, distFunc = 1, roiFunc = 1;
  double mortarThresh = 0.05;
  std::map<double, int> pdfs;  // cumulative Poisson probability -> # points (ConcurrentSkipListMap, put replaces)
};

// ---------------------------------------------------------------------------
// scene objects (mySceneObject.java:5-57)
struct SceneObject : GeomBase {
  bool inverted = false;
};
int GeomBase::shadowHit(Ray& ray, Ray& trans, const CTM* ctara, double d, uint64_t* st) {  // mySceneObject.java:33-38
  Hit h = intersect(ray, trans, ctara, st);
  if (h.isHit && (d - h.t) > EPS) return 1;
  return 0;
}

// planar objects (myPlanarObject.java). The reference flips vertex order in
// place when N.d > 0 (:110); both orientations are precomputed here and the one
// the mutation would produce is selected, which is the same function of
// (prim, ray) and keeps the oracle thread-safe.
struct PlanarState {
  std::vector<double> vx, vy, vz, vu, vv;
  std::vector<V3> P, P2P;
  V3 N, P2P0;
  double D = 0;
  std::vector<double> dotVals;
  double baryIDenom = 0;
};
struct Planar : SceneObject {
  int vCount = 3;
  bool isPlane = false;
  PlanarState st[2];  // [0] file order, [1] reversed
  std::vector<double> vx, vy, vz, vu, vv;
  static void set_points_and_normal(PlanarState& s, int vc) {  // :44-69
    s.P.assign(vc, V3());
    s.P2P.assign(vc, V3());
    s.dotVals.assign(vc + 1, 0);
    for (int i = 0; i < vc; i++) {
      s.P[i] = V3(s.vx[i], s.vy[i], s.vz[i]);
      int idx = (i != 0 ? i - 1 : vc - 1);
      s.P2P[idx] = V3(s.vx[i] - s.vx[idx], s.vy[i] - s.vy[idx], s.vz[i] - s.vz[idx]);
      s.dotVals[idx] = dot(s.P2P[idx], s.P2P[idx]);
    }
    s.P2P0 = s.P2P[2];
    s.P2P0 = V3(s.P2P0.x * -1.0, s.P2P0.y * -1.0, s.P2P0.z * -1.0);
    s.dotVals[vc] = -dot(s.P2P[0], s.P2P[2]);
    s.baryIDenom = 1.0 / ((s.dotVals[0] * s.dotVals[2]) - (s.dotVals[vc] * s.dotVals[vc]));
    s.N = cross(s.P2P[1], s.P2P[0]);
    normalize_ip(s.N);
  }
  static void set_eq(PlanarState& s) { s.D = -((s.N.x * s.vx[0]) + (s.N.y * s.vy[0]) + (s.N.z * s.vz[0])); }
  void finalize_poly();
  void build_reversed() {  // invertNormal :71-88
    PlanarState& a = st[0];
    PlanarState& b = st[1];
    int n = vCount;
    b.vx.assign(n, 0); b.vy.assign(n, 0); b.vz.assign(n, 0); b.vu.assign(n, 0); b.vv.assign(n, 0);
    for (int i = 0; i < n; i++) {
      b.vx[n - 1 - i] = a.vx[i]; b.vy[n - 1 - i] = a.vy[i]; b.vz[n - 1 - i] = a.vz[i];
      b.vu[n - 1 - i] = a.vu[i]; b.vv[n - 1 - i] = a.vv[i];
    }
    set_points_and_normal(b, n);
    set_eq(b);
  }
  virtual bool inside(const PlanarState& s, const V3& p) const {  // myTriangle/myQuad.checkInside :165-175,:200-211
    if (isPlane) return true;
    for (int i = 0; i < vCount; ++i) {
      int pIdx = (i == 0 ? vCount - 1 : i - 1);
      V3 ir(p.x - s.vx[i], p.y - s.vy[i], p.z - s.vz[i]);
      V3 tmp = cross(ir, s.P2P[pIdx]);
      if (dot(tmp, s.N) < -EPS) return false;
    }
    return true;
  }
  // selected orientation for a given transformed ray (intersectCheck :104-115)
  int pick(const Ray& tr, double& planeRes) const {
    planeRes = dot(st[0].N, tr.direction);
    if (!(std::fabs(planeRes) > 0)) return -1;
    if (planeRes > 0) {
      planeRes = dot(st[1].N, tr.direction);
      if (!(std::fabs(planeRes) > 0)) return -1;
      if (planeRes > 0) return -1;  // reference recurses forever (grazing non-planar quad)
      return 1;
    }
    return 0;
  }
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* stt) override {
    if (stt) stt[vCount == 3 && !isPlane ? ST_TRI : ST_QUAD]++;
    double planeRes;
    int s = pick(tr, planeRes);
    if (s < 0) return Hit();
    const PlanarState& S = st[s];
    double t = -(dot(S.N, tr.origin) + S.D) / planeRes;
    if ((t > EPS) && inside(S, tr.point(t))) {
      int args[2] = {s, 0};  // orientation travels with the hit (normal / texture lookups)
      return obj_hit(tr, this, ray.direction, ctara, tr.point(t), args, t);
    }
    return Hit();
  }
  V3 normalAt(const V3&, const int* args) override {  // :130-136
    V3 r = st[args ? args[0] : 0].N;
    normalize_ip(r);
    return r;
  }
  void txtrCoords(const V3& isct, const int* args, const Texture& tex, double, double& u, double& v) override {  // :178-186
    const PlanarState& S = st[args ? args[0] : 0];
    V3 v2 = vsub(isct, S.P[0]);
    double dot20 = dot(v2, S.P2P[0]), dot21 = dot(v2, S.P2P0);
    double c_u = ((S.dotVals[2] * dot20) - (S.dotVals[vCount] * dot21)) * S.baryIDenom;
    double c_v = ((S.dotVals[0] * dot21) - (S.dotVals[vCount] * dot20)) * S.baryIDenom;
    double c_w = 1 - c_u - c_v;
    double uu = S.vu[0] * c_w + S.vu[1] * c_u + S.vu[2] * c_v, vv2 = S.vv[0] * c_w + S.vv[1] * c_u + S.vv[2] * c_v;
    u = uu * (tex.w - 1);
    v = (1 - vv2) * (tex.h - 1);
  }
};

// implicit objects (myImpObject.java)
struct Sphere : SceneObject {
  double radX = 1, radY = 1, radZ = 1;
  bool moving = false;
  V3 origin0, origin1;
  V3 getOrigin(double t) override {  // :125, moving :153
    if (!moving) return origin;
    V3 bMa = vsub(origin1, origin0);
    return V3(origin0.x + t * bMa.x, origin0.y + t * bMa.y, origin0.z + t * bMa.z);
  }
  V3 orc(Ray& r) {  // originRadCalc :19-23
    V3 o = getOrigin(moving ? r.get_time() : 0);
    return V3((r.origin.x - o.x) / radX, (r.origin.y - o.y) / radY, (r.origin.z - o.z) / radZ);
  }
  double A(const Ray& r) const {
    return ((r.direction.x / radX) * (r.direction.x / radX)) + ((r.direction.y / radY) * (r.direction.y / radY)) +
           ((r.direction.z / radZ) * (r.direction.z / radZ));
  }
  double B(Ray& r) {
    V3 pC = orc(r);
    return 2 * (((r.direction.x / radX) * pC.x) + ((r.direction.y / radY) * pC.y) + ((r.direction.z / radZ) * pC.z));
  }
  double C(Ray& r) {
    V3 pC = orc(r);
    return (pC.x * pC.x) + (pC.y * pC.y) + (pC.z * pC.z) - 1;
  }
  V3 normalAt(const V3& pt, const int*) override {  // :68-74 (uses the static origin)
    V3 r(pt.x - origin.x, pt.y - origin.y, pt.z - origin.z);
    normalize_ip(r);
    if (inverted) r = V3(r.x * -1.0, r.y * -1.0, r.z * -1.0);
    return r;
  }
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {  // :76-94
    if (st) st[ST_SPHERE]++;
    double a = A(tr), ta = 2 * a, b = B(tr), c = C(tr), discr = ((b * b) - (2 * ta * c));
    if (!(discr < 0)) {
      double d1 = std::sqrt(discr), t1 = (-1 * b + d1) / (ta), t2 = (-1 * b - d1) / (ta);
      double tVal = jmin(t1, t2);
      if (tVal < EPS) {
        tVal = jmax(t1, t2);
        if (tVal < EPS) return Hit();
      }
      return obj_hit(tr, this, ray.direction, ctara, tr.point(tVal), nullptr, tVal);
    }
    return Hit();
  }
  void finalize_box() {  // L1 half-extent box :127-139
    double tv = radX + radY + radZ;
    minVals = V3(origin.x + -tv, origin.y + -tv, origin.z + -tv);
    maxVals = V3(origin.x + tv, origin.y + tv, origin.z + tv);
  }
  void txtrCoords(const V3& p, const int*, const Texture& tex, double time, double& u, double& v) override {  // :97-122
    V3 to = getOrigin(time);
    double a0 = p.y - to.y, a1 = a0 / radY;
    a1 = (a1 > 1) ? 1 : (a1 < -1) ? -1 : a1;
    v = (tex.h - 1) * jf::acos(a1) / M_PI;
    double shWm1 = tex.w - 1, z1 = p.z - to.z, q = v / (tex.h - 1);
    double b0 = (p.x - to.x) / radX;
    b0 = (b0 > 1) ? 1 : (b0 < -1) ? -1 : b0;
    double b1 = jf::sin(q * M_PI);
    double a2 = (std::fabs(b1) < EPS) ? 1 : b0 / b1;
    u = (z1 <= EPS) ? ((shWm1 * jf::acos(a2)) / TWO_PI_F + shWm1 / 2.0) : shWm1 - ((shWm1 * jf::acos(a2)) / TWO_PI_F + shWm1 / 2.0);
    u = (u < 0) ? 0 : (u > shWm1) ? shWm1 : u;
  }
};

struct HollowCyl : SceneObject {  // :157-237
  double radX = 1, radZ = 1, myHeight = 1, yTop = 1, yBottom = 0;
  double A(const Ray& r) const { return ((r.direction.x / radX) * (r.direction.x / radX)) + ((r.direction.z / radZ) * (r.direction.z / radZ)); }
  V3 orc(const Ray& r) const { return V3((r.origin.x - origin.x) / radX, (r.origin.y - origin.y) / 1.0, (r.origin.z - origin.z) / radZ); }
  double B(const Ray& r) const { V3 pC = orc(r); return 2 * (((r.direction.x / radX) * pC.x) + ((r.direction.z / radZ) * pC.z)); }
  double C(const Ray& r) const { V3 pC = orc(r); return (pC.x * pC.x) + (pC.z * pC.z) - 1; }
  void finalize_box() {
    double tv = radX + radZ;
    minVals = V3(origin.x + -tv, origin.y + 0, origin.z + -tv);
    maxVals = V3(origin.x + tv, origin.y + myHeight, origin.z + tv);
  }
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {
    if (st) st[ST_SPHERE]++;
    double a = A(tr), b = B(tr), c = C(tr), discr = ((b * b) - (4 * a * c));
    if (!(discr < 0)) {
      double d1 = std::sqrt(discr), t1 = (-b + d1) / (2 * a), t2 = (-b - d1) / (2 * a);
      double cv = jmin(t1, t2), co = jmax(t1, t2);
      if (cv < -EPS) {
        double tmp = co; co = cv; cv = tmp;
        if (cv < -EPS) return Hit();
      }
      double y1 = tr.origin.y + (cv * tr.direction.y);
      if ((cv > EPS) && (y1 > yBottom) && (y1 < yTop)) { int a0[2] = {0, 0}; return obj_hit(tr, this, ray.direction, ctara, tr.point(cv), a0, cv); }
      double y2 = tr.origin.y + (co * tr.direction.y);
      if ((co > EPS) && (y2 > yBottom) && (y2 < yTop)) { int a1[2] = {1, 0}; return obj_hit(tr, this, ray.direction, ctara, tr.point(co), a1, co); }
    }
    return Hit();
  }
  V3 normalAt(const V3& pt, const int* args) override {
    V3 r = (args[0] == 1) ? V3(origin.x - pt.x, 0, origin.z - pt.z) : V3(pt.x - origin.x, 0, pt.z - origin.z);
    normalize_ip(r);
    if (inverted) r = V3(r.x * -1, r.y * -1, r.z * -1);
    return r;
  }
};
struct Cyl : HollowCyl {  // :239-327
  double cap[2][4];
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {
    if (st) st[ST_SPHERE]++;
    double a = A(tr), b = B(tr), c = C(tr);
    double discr = ((b * b) - (4 * a * c));
    if (!(discr < 0)) {
      double d1 = std::sqrt(discr), t1 = (-b + d1) / (2 * a), t2 = (-b - d1) / (2 * a);
      double cv = jmin(t1, t2), co = jmax(t1, t2);
      if (cv < EPS) {
        co = cv;
        cv = jmax(t1, t2);
        if (cv < EPS) return Hit();
      }
      bool planeRes = true;
      double num[2] = {0, 0}, den[2] = {1, 1}, pl[2] = {0, 0};
      for (int i = 0; i < 2; ++i) {
        den[i] = cap[i][0] * tr.direction.x + cap[i][1] * tr.direction.y + cap[i][2] * tr.direction.z;
        if (std::fabs(den[i]) > EPS) {
          num[i] = cap[i][0] * tr.origin.x + cap[i][1] * tr.origin.y + cap[i][2] * tr.origin.z + cap[i][3];
          pl[i] = -num[i] / den[i];
        } else pl[i] = 10000;
      }
      double pltVal = jmin(pl[0], pl[1]);
      int idxVis = (pltVal == pl[0] ? 0 : 1);
      if (pltVal < 0) {
        pltVal = pl[idxVis];
        if (pltVal < EPS) planeRes = false;
      }
      double tVal = 0, maxT = jmax(cv, co), minT = jmin(cv, co);
      if (planeRes && (((minT <= 0) && (pltVal >= -EPS) && (pltVal <= maxT)) || ((pltVal > minT) && (pltVal <= maxT)))) {
        tVal = pltVal;
      } else {
        tVal = cv;
        idxVis = 2;
      }
      double y1 = tr.origin.y + (tVal * tr.direction.y);
      if ((y1 + EPS >= yBottom) && (y1 - EPS <= yTop)) { int ar[2] = {idxVis, 0}; return obj_hit(tr, this, ray.direction, ctara, tr.point(tVal), ar, tVal); }
    }
    return Hit();
  }
  V3 normalAt(const V3& pt, const int* args) override {
    V3 r = (args[0] >= 2) ? V3(pt.x - origin.x, 0, pt.z - origin.z) : V3(cap[args[0]][0], cap[args[0]][1], cap[args[0]][2]);
    normalize_ip(r);
    if (inverted) r = V3(r.x * -1, r.y * -1, r.z * -1);
    return r;
  }
};

// myRndrdBox (mySceneObject.java:59-92): the bbox intersection, rendered
struct RndrdBox : SceneObject {
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override { return bbox->intersect(ray, tr, ctara, st); }
  V3 normalAt(const V3& pt, const int* args) override { return bbox->normalAt(pt, args); }
};

// ---------------------------------------------------------------------------
// lights (myLight.java)
enum LightType { LT_POINT = 0, LT_SPOT = 1, LT_DISK = 2 };
struct Light : SceneObject {
  int ltype = LT_POINT;
  Color lightColor;
  V3 orientation;
  double innerRad = 0, outerRad = 0, radDiff = 0;
  V3 oPhAxis;
  double radius = 0;
  V3 surfTangent;
  int index = 0;  // position in lightList
  V3 disk_pos(const RKey& k, uint32_t kk) const {  // getRandomDiskPos :251-258
    V3 tmp = rot_around_axis(surfTangent, orientation,
                             rng_range(rng_bits(k.seed, k.pixel, k.sample, k.node, SITE_DISK + index, kk), 0, TWO_PI_F));
    normalize_ip(tmp);
    double m = rng_range(rng_bits(k.seed, k.pixel, k.sample, k.node, SITE_DISK + index, kk + 1), 0, radius);
    tmp = V3(tmp.x * m, tmp.y * m, tmp.z * m);
    return V3(tmp.x + origin.x, tmp.y + origin.y, tmp.z + origin.z);
  }
  Hit intersect(Ray&, Ray&, const CTM*, uint64_t*) override { return Hit(); }
  V3 normalAt(const V3&, const int*) override { return V3(0, 1, 0); }
  double angle_prob(double angle) const {  // :77
    return (angle < innerRad) ? 1 : (angle > outerRad) ? 0 : (outerRad - angle) / radDiff;
  }
};

// ---------------------------------------------------------------------------
// accel structures (myGeomBase.java:200-423)
struct GeomList;
struct AccelStruct : GeomBase {
  bool isAccel() const override { return true; }
  virtual Hit traverse(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) = 0;
  Hit intersect(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {  // :216-222
    Hit bh = bbox->slab_hit(tr, st);
    if (!bh.isHit) return bh;
    return traverse(ray, tr, ctara, st);
  }
  V3 normalAt(const V3& p, const int* a) override { return bbox->normalAt(p, a); }
  V3 getMaxVec() override { return bbox->maxVals; }  // :240-243
  V3 getMinVec() override { return bbox->minVals; }
};
struct GeomList : AccelStruct {  // :251-306
  std::vector<GeomBase*> objs;
  void add_obj(GeomBase* o);
  int shadowHit(Ray& ray, Ray& tr, const CTM* ctara, double d, uint64_t* st) override {
    if (bbox->shadowHit(ray, tr, ctara, d, st) == 0) return 0;
    for (GeomBase* o : objs) {
      Ray otr = transformed(ray, o->ctm->inv, o->key);
      if (o->shadowHit(ray, otr, ctara, d, st) == 1) return 1;
    }
    return 0;
  }
  Hit traverse(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {
    double clsT = DMAX;
    Hit cls;
    bool have = false;
    GeomBase* clsObj = nullptr;
    Ray clsTr;
    for (GeomBase* o : objs) {
      Ray otr = transformed(ray, o->ctm->inv, o->key);
      Hit h = o->intersect(ray, otr, o->ctm.get(), st);
      if (h.t < clsT) {
        clsObj = o; cls = h; clsT = h.t; clsTr = otr; have = true;
      }
    }
    if (!have) return Hit();
    // reCalcCTMHitNorm(reBuildCTMara(objCTM, listCTM)) (myRay.java:168-175): Q4 double transform
    auto nc = std::make_shared<CTM>(build_ctm(mmul(ctm->g, clsObj->ctm->g)));
    cls.ctm_own = nc;
    cls.ctm = nc.get();
    cls.fwdTransHitLoc = xpt(nc->g, cls.hitLoc);
    if (clsObj->isAccel()) {  // nested accel (not on the config path)
      return static_cast<AccelStruct*>(clsObj)->traverse(ray, clsTr, cls.ctm, st);
    }
    V3 n = cls.obj->normalAt(cls.hitLoc, cls.args);  // rayHit.obj: the primitive, also through an instance
    n = xvec(nc->adj, n);
    normalize_ip(n);
    cls.objNorm = n;
    return cls;
  }
};
struct BVH : AccelStruct {  // :309-423
  bool isLeaf = true;
  GeomList* leafVals = nullptr;
  BVH *left = nullptr, *right = nullptr;
  int depth = 0;
  int shadowHit(Ray& ray, Ray& tr, const CTM* ctara, double d, uint64_t* st) override {
    if (isLeaf) return leafVals->shadowHit(ray, tr, ctara, d, st);
    int lr = left->bbox->shadowHit(ray, tr, ctara, d, st);
    if ((lr == 1) && left->shadowHit(ray, tr, ctara, d, st) == 1) return 1;
    int rr = right->bbox->shadowHit(ray, tr, ctara, d, st);
    if ((rr == 1) && right->shadowHit(ray, tr, ctara, d, st) == 1) return 1;
    return 0;
  }
  Hit traverse(Ray& ray, Ray& tr, const CTM* ctara, uint64_t* st) override {
    if (isLeaf) return leafVals->traverse(ray, tr, ctara, st);
    Hit h = left->bbox->slab_hit(tr, st);
    if (h.isHit) h = left->traverse(ray, tr, ctara, st);
    Hit h2 = right->bbox->slab_hit(tr, st);
    if (h2.isHit && (!h.isHit || (h2.t < h.t))) h2 = right->traverse(ray, tr, ctara, st);
    return h.t <= h2.t ? h : h2;
  }
};

// myInstance (mySceneObject.java:95-145): the named object tested with the instance's
// transformed ray as both of its rays (so an instanced accel re-normalises that ray in
// place and tests its boxes with it) and the instance CTM array; the instance shader
// (`instance <name> shdr`) replaces the hit's. Hits keep the primitive as rayHit.obj.
struct Instance : GeomBase {
  GeomBase* obj = nullptr;
  bool useShader = false;
  Hit intersect(Ray&, Ray& tr, const CTM* ctara, uint64_t* st) override {
    Hit h = obj->intersect(tr, tr, ctara, st);
    if (useShader) h.shdr = shdr;
    return h;
  }
  int shadowHit(Ray&, Ray& tr, const CTM* ctara, double d, uint64_t* st) override {
    return obj->shadowHit(tr, tr, ctara, d, st);
  }
  V3 normalAt(const V3& p, const int* a) override { return obj->normalAt(p, a); }
  V3 getOrigin(double t) override { return xpt(obj->ctm->g, obj->getOrigin(t)); }
  V3 getMaxVec() override { return xpt(obj->ctm->g, obj->getMaxVec()); }
  V3 getMinVec() override { return xpt(obj->ctm->g, obj->getMinVec()); }
};

// ---------------------------------------------------------------------------
// photon map (myLight.java:278-446)
struct Photon {
  double pwr[3];
  double pos[4];
};
struct KDNode {
  int photon = -1;
  int axis = -1;
  int left = -1, right = -1;
};
struct KDTree {
  std::vector<Photon> photons;
  std::vector<KDNode> nodes;
  int root = -1;
  int num_Cast = 0, maxNear = 0;
  double baseMaxDist2 = 0;
  int build(std::vector<int>& idx, int lo, int hi) {  // build_tree :332-381 on idx[lo,hi)
    KDNode n;
    int sz = hi - lo;
    if (sz == 1) {
      n.photon = idx[lo];
      n.axis = -1;
      nodes.push_back(n);
      return (int)nodes.size() - 1;
    }
    double mins[3] = {1e20, 1e20, 1e20}, maxs[3] = {-1e20, -1e20, -1e20};
    for (int i = lo; i < hi; i++) {
      const Photon& p = photons[idx[i]];
      for (int j = 0; j < 3; j++) {
        if (p.pos[j] < mins[j]) mins[j] = p.pos[j];
        if (p.pos[j] > maxs[j]) maxs[j] = p.pos[j];
      }
    }
    double dx = maxs[0] - mins[0], dy = maxs[1] - mins[1], dz = maxs[2] - mins[2];
    int ax = 2;
    if (dx >= dy && dx >= dz) ax = 0;
    else if (dy >= dx && dy >= dz) ax = 1;
    // Collections.sort: stable, comparator with 0 on equality
    std::stable_sort(idx.begin() + lo, idx.begin() + hi, [&](int a, int b) { return photons[a].pos[ax] < photons[b].pos[ax]; });
    int split = sz / 2;
    n.photon = idx[lo + split];
    n.axis = ax;
    int me = (int)nodes.size();
    nodes.push_back(n);
    int l = -1, r = -1;
    if (split != 0) l = build(idx, lo, lo + split);
    if (split != sz - 1) r = build(idx, lo + split + 1, hi);
    nodes[me].left = l;
    nodes[me].right = r;
    return me;
  }
  void build_all() {
    nodes.clear();
    root = -1;
    if (photons.empty()) return;
    std::vector<int> idx(photons.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    nodes.reserve(photons.size());
    root = build(idx, 0, (int)idx.size());
  }
  struct QE {
    double d2;
    int p;
  };
  // java.util.PriorityQueue<myPhoton>(n, Collections.reverseOrder()) as JDK 8 implements it
  // (offer -> siftUpUsingComparator, poll -> siftDownUsingComparator; the comparator is
  // myPhoton.compareTo on pos[3] = d2, reversed: a max-heap). An element moves up only past a
  // STRICTLY smaller parent and down only past a STRICTLY larger child (the right child only when
  // strictly larger than the left), so among photons of equal d2 the one poll() evicts and the
  // poll order of the sum are Java's -- std::priority_queue's sifts break ties differently.
  struct JavaMaxPQ {
    std::vector<QE> q;
    size_t size() const { return q.size(); }
    bool empty() const { return q.empty(); }
    const QE& peek() const { return q[0]; }
    void add(const QE& x) {  // offer + siftUp
      size_t k = q.size();
      q.push_back(x);
      while (k > 0) {
        const size_t parent = (k - 1) >> 1;
        if (q[parent].d2 >= x.d2) break;  // reverseOrder.compare(x, e) >= 0
        q[k] = q[parent];
        k = parent;
      }
      q[k] = x;
    }
    QE poll() {  // the root; the last element sifts down from the root
      const QE r = q[0];
      const QE x = q.back();
      q.pop_back();
      const size_t n = q.size();
      if (n > 0) {
        size_t k = 0;
        const size_t half = n >> 1;
        while (k < half) {
          size_t child = 2 * k + 1;
          const size_t right = child + 1;
          if (right < n && q[right].d2 > q[child].d2) child = right;  // compare(c, right) > 0
          if (x.d2 >= q[child].d2) break;                              // compare(x, c) <= 0
          q[k] = q[child];
          k = child;
        }
        q[k] = x;
      }
      return r;
    }
  };
  void near_rec(const double pos[3], int ni, JavaMaxPQ& q, double& max_d2, uint64_t* st) const {  // :408-445
    const KDNode& n = nodes[ni];
    const Photon& ph = photons[n.photon];
    if (st) st[ST_PHOTON]++;
    if (n.axis != -1) {
      double delta = pos[n.axis] - ph.pos[n.axis], delta2 = delta * delta;
      if (delta < 0) {
        if (n.left != -1) near_rec(pos, n.left, q, max_d2, st);
        if (n.right != -1 && delta2 < max_d2) near_rec(pos, n.right, q, max_d2, st);
      } else {
        if (n.right != -1) near_rec(pos, n.right, q, max_d2, st);
        if (n.left != -1 && delta2 < max_d2) near_rec(pos, n.left, q, max_d2, st);
      }
    }
    double dx = pos[0] - ph.pos[0], dy = pos[1] - ph.pos[1], dz = pos[2] - ph.pos[2];
    double len2 = dx * dx + dy * dy + dz * dz;
    if (len2 < max_d2) {
      q.add(QE{len2, n.photon});
      if ((int)q.size() > maxNear) q.poll();  // delete the most distant photon
      if ((int)q.size() == maxNear) {
        if (q.peek().d2 < max_d2) max_d2 = q.peek().d2;
      }
    }
  }
  // find_near (:389-405): the neighbourhood in poll order (farthest first)
  void find_near(const V3& p, std::vector<QE>& out, uint64_t* st) const {
    out.clear();
    if (root < 0) return;
    JavaMaxPQ q;
    double max_d2 = baseMaxDist2;
    const double pos[3] = {p.x, p.y, p.z};
    near_rec(pos, root, q, max_d2, st);
    while (!q.empty()) out.push_back(q.poll());
  }
  // getIrradianceFromPhtnTree (myObjShader.java:441-458)
  void irradiance(const V3& p, double res[3], uint64_t* st) const {
    res[0] = res[1] = res[2] = 0;
    std::vector<QE> order;
    find_near(p, order, st);
    if (order.empty()) return;  // [null] -> zero (Q20)
    double rSq = order[0].d2;   // hood.get(0): the farthest
    double area = PI_F * rSq;
    for (const QE& e : order) {  // the reference sums in poll order (farthest first)
      res[0] += photons[e.p].pwr[0];
      res[1] += photons[e.p].pwr[1];
      res[2] += photons[e.p].pwr[2];
    }
    res[0] /= area; res[1] /= area; res[2] /= area;
  }
};

// ---------------------------------------------------------------------------
struct Scene {
  std::vector<std::unique_ptr<GeomBase>> owned;
  std::vector<std::unique_ptr<Shader>> shaders;
  std::vector<GeomBase*> objList;
  std::vector<Light*> lightList;
  int W = 300, H = 300;
  int numRaysPerPixel = 0;
  int numRays = 8, numPhotonRays = 4;
  double fov = 60, viewZ = -1;
  // camera: 0 myFOVScene, 1 myFishEyeScene (fishEye degrees), 2 myOrthoScene (width, height)
  int camType = 0;
  double fishEye = 0, orthoW = 0, orthoH = 0;
  Color backgroundColor;
  bool txtrdBkg = false;
  Sphere* skyDome = nullptr;
  const Texture* bkgTex = nullptr;
  bool hasDOF = false;
  double lensRadius = 0, lensFocal = 0;
  Planar* focalPlane = nullptr;
  bool usePhotonMap = false, isCausticPhtn = false, photonsBuilt = false;
  KDTree photonTree;
  double causticsLightPwrMult = 40.0, diffuseLightPwrMult = 8.0;
  uint32_t primCount = 0;
  std::map<std::string, Texture>* textures = nullptr;
  // BVH statistics
  long bvhInternal = 0, bvhLeaves = 0;
  int bvhDepth = 0;
  long bvhPrims = 0;

  template <class T>
  T* make() {
    T* p = new T();
    p->scene = this;
    owned.emplace_back(p);
    return p;
  }
};

BBox::BBox(Scene* s, const V3& mn, const V3& mx) {
  scene = s;
  calc_min_max(mn, mx);
}
static BBox* make_bbox(Scene* s, GeomBase* owner) {  // postProcBBox (myGeomBase.java:42-45)
  BBox* b = new BBox(s, owner->minVals, owner->maxVals);
  s->owned.emplace_back(b);
  b->add_obj(owner);
  owner->bbox = b;
  return b;
}
// expandBoxPt / expandBoxByBox (DistRayTracer.java:353-371)
static void expand_pt(BBox* b, const V3& p) {
  b->minVals.x = (b->minVals.x < p.x) ? b->minVals.x : p.x;
  b->minVals.y = (b->minVals.y < p.y) ? b->minVals.y : p.y;
  b->minVals.z = (b->minVals.z < p.z) ? b->minVals.z : p.z;
  b->maxVals.x = (b->maxVals.x > p.x) ? b->maxVals.x : p.x;
  b->maxVals.y = (b->maxVals.y > p.y) ? b->maxVals.y : p.y;
  b->maxVals.z = (b->maxVals.z > p.z) ? b->maxVals.z : p.z;
}
static void expand_box(BBox* t, BBox* s, const M4* fwd) {
  if (fwd) {
    expand_pt(t, xpt(*fwd, s->minVals));
    expand_pt(t, xpt(*fwd, s->maxVals));
  } else {
    expand_pt(t, s->minVals);
    expand_pt(t, s->maxVals);
  }
}
void GeomList::add_obj(GeomBase* o) {  // myGeomBase.java:261-266
  objs.push_back(o);
  M4 tmp = mmul(ctm->inv, o->ctm->g);
  expand_box(bbox, o->bbox, &tmp);
}
void Planar::finalize_poly() {  // :93-100
  st[0].vx = vx; st[0].vy = vy; st[0].vz = vz; st[0].vu = vu; st[0].vv = vv;
  set_points_and_normal(st[0], vCount);
  set_eq(st[0]);
  double sx = 0, sy = 0, sz = 0;
  for (int i = 0; i < vCount; ++i) { sx += vx[i]; sy += vy[i]; sz += vz[i]; }
  origin = V3(sx / vCount, sy / vCount, sz / vCount);
  trans_origin = xpt(ctm->g, origin);
  double mnx = DMAX, mny = DMAX, mnz = DMAX, mxx = -DMAX, mxy = -DMAX, mxz = -DMAX;
  for (int i = 0; i < vCount; ++i) {
    if (vx[i] < mnx) mnx = vx[i]; if (vy[i] < mny) mny = vy[i]; if (vz[i] < mnz) mnz = vz[i];
    if (vx[i] > mxx) mxx = vx[i]; if (vy[i] > mxy) mxy = vy[i]; if (vz[i] > mxz) mxz = vz[i];
  }
  minVals = V3(mnx, mny, mnz);
  maxVals = V3(mxx, mxy, mxz);
  bbox->calc_min_max(minVals, maxVals);
  bbox->add_obj(this);
  build_reversed();
}

// ---------------------------------------------------------------------------
// BVH build (myScene.java:305-324, myGeomBase.java:329-386, DistRayTracer.java:409-418)
typedef std::vector<GeomBase*> OList;
static OList sorted_by(const OList& in, int axis) {
  OList r(in);
  std::stable_sort(r.begin(), r.end(), [axis](GeomBase* a, GeomBase* b) {
    return jdcompare(comp(a->trans_origin, axis), comp(b->trans_origin, axis)) < 0;
  });
  return r;
}
static void build_sorted(const OList& src, int skip, OList out[3]) {  // buildSortedObjAras :338-357
  for (int i = 0; i < 3; ++i) {
    if (i == skip) out[i] = src;
    else out[i] = sorted_by(src, i);
  }
}
static int max_span_idx(OList l[3]) {
  double maxSpan = -1;
  int idx = -1;
  size_t n = l[0].size();
  for (int i = 0; i < 3; ++i) {
    double diff = comp(l[i][n - 1]->trans_origin, i) - comp(l[i][0]->trans_origin, i);
    if (maxSpan < diff) { maxSpan = diff; idx = i; }
  }
  return idx;
}
static BVH* new_bvh(Scene* s, std::shared_ptr<CTM> c) {  // myBVH ctor :318-327
  BVH* b = s->make<BVH>();
  b->ctm = c;
  GeomList* gl = s->make<GeomList>();
  gl->ctm = c;
  make_bbox(s, gl);
  b->leafVals = gl;
  make_bbox(s, b);
  return b;
}
static void add_obj_list(Scene* s, BVH* node, OList lists[3], int stIDX, int endIDX) {  // :360-386
  int sz = endIDX - stIDX;
  if (sz <= 5) {
    node->isLeaf = true;
    GeomList* gl = s->make<GeomList>();
    gl->ctm = node->ctm;
    make_bbox(s, gl);
    for (GeomBase* o : lists[0]) gl->add_obj(o);
    node->leafVals = gl;
    expand_box(node->bbox, gl->bbox, nullptr);
    s->bvhLeaves++;
    s->bvhPrims += (long)lists[0].size();
    if (node->depth > s->bvhDepth) s->bvhDepth = node->depth;
  } else {
    node->isLeaf = false;
    s->bvhInternal++;
    int split = (int)(.5 * sz);
    int ax = max_span_idx(lists);
    node->left = new_bvh(s, node->ctm);
    node->right = new_bvh(s, node->ctm);
    node->left->depth = node->right->depth = node->depth + 1;
    OList lsub(lists[ax].begin(), lists[ax].begin() + split);
    OList rsub(lists[ax].begin() + split, lists[ax].begin() + sz);
    OList ll[3], rl[3];
    build_sorted(lsub, ax, ll);
    build_sorted(rsub, ax, rl);
    add_obj_list(s, node->left, ll, stIDX, stIDX + split);
    add_obj_list(s, node->right, rl, stIDX + split, endIDX);
    expand_box(node->bbox, node->left->bbox, nullptr);
    expand_box(node->bbox, node->right->bbox, nullptr);
  }
}

// ---------------------------------------------------------------------------
// ray core (myScene.java:879-914)
static Color shade(Scene* s, Hit& hit, uint64_t* st);
static Color background(Scene* s, Ray& ray, uint64_t* st);

static int calc_shadow(Scene* s, Ray& ray, double d, uint64_t* st) {  // :879-885
  for (GeomBase* o : s->objList) {
    Ray tr = transformed(ray, o->ctm->inv, o->key);
    if (o->shadowHit(ray, tr, o->ctm.get(), d, st) == 1) return 1;
  }
  return 0;
}
static Hit closest_hit(Scene* s, Ray& ray, uint64_t* st) {  // :888-903 (TreeMap: first inserted wins ties)
  Hit best;
  for (GeomBase* o : s->objList) {
    Ray tr = transformed(ray, o->ctm->inv, o->key);
    Hit h = o->intersect(ray, tr, o->ctm.get(), st);
    if (h.isHit && h.t < best.t) best = h;
  }
  return best;
}
static Color reflect_ray(Scene* s, Ray& ray, uint64_t* st) {  // :907-914
  Hit h = closest_hit(s, ray, st);
  if (h.isHit) return shade(s, h, st);
  if (s->txtrdBkg) return background(s, ray, st);
  return s->backgroundColor;
}

// skydome (myScene.java:1104-1149)
static Color background(Scene* s, Ray& ray, uint64_t* st) {
  Sphere* sd = s->skyDome;
  const Texture& tex = *s->bkgTex;
  double a = sd->A(ray), b = sd->B(ray), c = sd->C(ray);
  double discr = ((b * b) - (4 * a * c));
  double t = -DMAX;
  if (discr > 0) {
    double d1 = std::sqrt(discr), t1 = (-1 * b + d1) / (2 * a), t2 = (-1 * b - d1) / (2 * a), tv = jmin(t1, t2);
    if (tv < EPS) tv = jmax(t1, t2);
    t = tv;
  }
  V3 p = ray.point(t);
  double a0 = p.y - sd->origin.y, a1 = a0 / (sd->radY);
  a1 = (a1 > 1) ? 1 : (a1 < -1) ? -1 : a1;
  double v = (tex.h - 1) * jf::acos(a1) / M_PI;
  double shWm1 = tex.w - 1, z1 = (p.z - sd->origin.z), q = v / (tex.h - 1);
  double b0 = (p.x - sd->origin.x) / (sd->radX);
  b0 = (b0 > 1) ? 1 : (b0 < -1) ? -1 : b0;
  double b1 = jf::sin(q * M_PI);
  double a2 = (std::fabs(b1) < EPS) ? 1 : b0 / b1;
  double u = (z1 <= EPS) ? ((shWm1 * (jf::acos(a2)) / (TWO_PI_F)) + shWm1 / 2.0) : shWm1 - ((shWm1 * (jf::acos(a2)) / (TWO_PI_F)) + shWm1 / 2.0);
  u = (u < 0) ? 0 : (u > shWm1) ? shWm1 : u;
  if (st) st[ST_TEXEL]++;
  long idx = (long)jd2i(v) * tex.w + jd2i(u);
  if (idx < 0) idx = 0;
  if (idx >= (long)tex.px.size()) idx = (long)tex.px.size() - 1;
  return color_from_int(tex.px[idx]);
}

// Perlin noise (float) DistRayTracer.java:234-310
static const int PERM_P[256] = {151,160,137,91,90,15,131,13,201,95,96,53,194,233,7,225,140,36,103,30,69,142,8,99,37,240,21,10,23,
  190,6,148,247,120,234,75,0,26,197,62,94,252,219,203,117,35,11,32,57,177,33,88,237,149,56,87,174,20,125,136,171,168,68,175,74,165,71,
  134,139,48,27,166,77,146,158,231,83,111,229,122,60,211,133,230,220,105,92,41,55,46,245,40,244,102,143,54,65,25,63,161,1,216,80,73,209,
  76,132,187,208,89,18,169,200,196,135,130,116,188,159,86,164,100,109,198,173,186,3,64,52,217,226,250,124,123,5,202,38,147,118,126,255,
  82,85,212,207,206,59,227,47,16,58,17,182,189,28,42,223,183,170,213,119,248,152,2,44,154,163,70,221,153,101,155,167,43,172,9,129,22,39,
  253,19,98,108,110,79,113,224,232,178,185,112,104,218,246,97,228,251,34,242,193,238,210,144,12,191,179,162,241,81,51,145,235,249,14,239,
  107,49,192,214,31,181,199,106,157,184,84,204,176,115,121,50,45,127,4,150,254,138,236,205,93,222,114,67,29,24,72,243,141,128,195,78,66,
  215,61,156,180};
static const int GRAD3[12][3] = {{1,1,0},{-1,1,0},{1,-1,0},{-1,-1,0},{1,0,1},{-1,0,1},{1,0,-1},{-1,0,-1},{0,1,1},{0,-1,1},{0,1,-1},{0,-1,-1}};
static inline int perm(int i) { return PERM_P[i & 255]; }
static inline int ffloor(float x) { return x > 0 ? (int)x : (int)x - 1; }
static inline float gdot(const int* g, float x, float y, float z) { return g[0] * x + g[1] * y + g[2] * z; }
static inline float fmix(float a, float b, float t) { return (1 - t) * a + t * b; }
static inline float fade(float t) { return t * t * t * (t * (t * 6 - 15) + 10); }
static float noise3(float x, float y, float z) {
  int X = ffloor(x), Y = ffloor(y), Z = ffloor(z);
  x = x - X; y = y - Y; z = z - Z;
  X = X & 255; Y = Y & 255; Z = Z & 255;
  int gi000 = perm(X + perm(Y + perm(Z))) % 12, gi001 = perm(X + perm(Y + perm(Z + 1))) % 12;
  int gi010 = perm(X + perm(Y + 1 + perm(Z))) % 12, gi011 = perm(X + perm(Y + 1 + perm(Z + 1))) % 12;
  int gi100 = perm(X + 1 + perm(Y + perm(Z))) % 12, gi101 = perm(X + 1 + perm(Y + perm(Z + 1))) % 12;
  int gi110 = perm(X + 1 + perm(Y + 1 + perm(Z))) % 12, gi111 = perm(X + 1 + perm(Y + 1 + perm(Z + 1))) % 12;
  float n000 = gdot(GRAD3[gi000], x, y, z), n100 = gdot(GRAD3[gi100], x - 1, y, z);
  float n010 = gdot(GRAD3[gi010], x, y - 1, z), n110 = gdot(GRAD3[gi110], x - 1, y - 1, z);
  float n001 = gdot(GRAD3[gi001], x, y, z - 1), n101 = gdot(GRAD3[gi101], x - 1, y, z - 1);
  float n011 = gdot(GRAD3[gi011], x, y - 1, z - 1), n111 = gdot(GRAD3[gi111], x - 1, y - 1, z - 1);
  float u = fade(x), v = fade(y), w = fade(z);
  return fmix(fmix(fmix(n000, n100, u), fmix(n010, n110, u), v), fmix(fmix(n001, n101, u), fmix(n011, n111, u), v), w);
}

// texture handlers (myTextureHandler.java)
static void image_color(Hit& hit, const Texture& tex, double out[3], uint64_t* st) {  // :84-103
  double u, v;
  double time = 0;
  if (Sphere* sp = dynamic_cast<Sphere*>(hit.obj)) { if (sp->moving) time = hit.transRay.get_time(); }
  hit.obj->txtrCoords(hit.hitLoc, hit.args, tex, time, u, v);
  int uInt = jd2i(u), vInt = jd2i(v);
  long idx00 = (long)vInt * tex.w + uInt, idx10 = idx00 + tex.w, idx01 = idx00 + 1, idx11 = idx10 + 1;
  long n = (long)tex.px.size();
  auto at = [&](long i) { if (i < 0) i = 0; if (i >= n) i = n - 1; return color_from_int(tex.px[i]); };
  if (st) st[ST_TEXEL]++;
  Color c00 = at(idx00), c10 = at(idx10), c01 = at(idx01), c11 = at(idx11);
  double fu = u - uInt, fv = v - vInt;
  auto lerp = [](const Color& a, double t, const Color& b) { return Color(a.r + t * (b.r - a.r), a.g + t * (b.g - a.g), a.b + t * (b.b - a.b)); };
  Color c0 = lerp(c00, fu, c01), c1 = lerp(c10, fu, c11), c = lerp(c0, fv, c1);
  out[0] = c.r; out[1] = c.g; out[2] = c.b;
}
static void clr_ara(const Shader* sh, double distVal, const V3& raw, double res[3], int i0 = 0, int i1 = 1) {  // getClrAra :277-294
  V3 pt(raw.x * sh->colorScale, raw.y * sh->colorScale, raw.z * sh->colorScale);
  double mult = sh->colorMult;
  double rm[3] = {1.0, 1.0, 1.0};
  if (sh->rndColors) {
    rm[0] = 1.0 + (mult * noise3((float)pt.x, (float)pt.z, (float)pt.y));
    rm[1] = 1.0 + (mult * noise3((float)pt.y, (float)pt.x, (float)pt.z));
    rm[2] = 1.0 + (mult * noise3((float)pt.z, (float)pt.y, (float)pt.x));
  }
  const Color &c0 = sh->colors.at(i0), &c1 = sh->colors.at(i1);
  res[0] = jmax(0, jmin(1.0, (c0.r) + rm[0] * distVal * ((c1.r) - (c0.r))));
  res[1] = jmax(0, jmin(1.0, (c0.g) + rm[1] * distVal * ((c1.g) - (c0.g))));
  res[2] = jmax(0, jmin(1.0, (c0.b) + rm[2] * distVal * ((c1.b) - (c0.b))));
}
// DistRayTracer.getClr (DistRayTracer.java:467-530): the named colours of noise_color
// (clr_rnd draws from Processing's unseeded random and is not supported)
static bool named_color(std::string n, Color& c) {
  for (auto& ch : n) ch = (char)std::tolower(ch);
  static const std::map<std::string, V3> tab = {
      {"clr_gray", V3(0.47, 0.47, 0.47)}, {"clr_white", V3(1.0, 1.0, 1.0)}, {"clr_yellow", V3(1.0, 1.0, 0)},
      {"clr_cyan", V3(0, 1.0, 1.0)}, {"clr_magenta", V3(1.0, 0, 1.0)}, {"clr_red", V3(1.0, 0, 0)},
      {"clr_blue", V3(0, 0, 1.0)}, {"clr_purple", V3(0.6, 0.2, 1.0)}, {"clr_green", V3(0, 1.0, 0)},
      {"clr_ltwood1", V3(0.94, 0.47, 0.12)}, {"clr_ltwood2", V3(0.94, 0.8, 0.4)}, {"clr_dkwood1", V3(0.2, 0.08, 0.08)},
      {"clr_dkwood2", V3(0.3, 0.20, 0.16)}, {"clr_mortar1", V3(0.2, 0.2, 0.2)}, {"clr_mortar2", V3(0.7, 0.7, 0.7)},
      {"clr_brick1_1", V3(0.6, 0.18, 0.22)}, {"clr_brick1_2", V3(0.8, 0.26, 0.33)}, {"clr_brick2_1", V3(0.6, 0.32, 0.16)},
      {"clr_brick2_2", V3(0.8, 0.45, 0.25)}, {"clr_brick3_1", V3(0.3, 0.01, 0.07)}, {"clr_brick3_2", V3(0.6, 0.02, 0.13)},
      {"clr_brick4_1", V3(0.4, 0.1, 0.17)}, {"clr_brick4_2", V3(0.6, 0.3, 0.13)}, {"clr_darkgray", V3(0.31, 0.31, 0.31)},
      {"clr_darkred", V3(0.47, 0, 0)}, {"clr_darkblue", V3(0, 0, 0.47)}, {"clr_darkpurple", V3(0.4, 0.2, 0.6)},
      {"clr_darkgreen", V3(0, 0.47, 0)}, {"clr_darkyellow", V3(0.47, 0.47, 0)}, {"clr_darkmagenta", V3(0.47, 0, 0.47)},
      {"clr_darkcyan", V3(0, 0.47, 0.47)}, {"clr_lightgray", V3(0.78, 0.78, 0.78)}, {"clr_lightred", V3(1.0, .43, .43)},
      {"clr_lightblue", V3(0.43, 0.43, 1.0)}, {"clr_lightgreen", V3(0.43, 1.0, 0.43)}, {"clr_lightyellow", V3(1.0, 1.0, .43)},
      {"clr_lightmagenta", V3(1.0, .43, 1.0)}, {"clr_lightcyan", V3(0.43, 1.0, 1.0)}, {"clr_black", V3(0, 0, 0)},
      {"clr_nearblack", V3(0.05, 0.05, 0.05)}, {"clr_faintgray", V3(0.43, 0.43, 0.43)}, {"clr_faintred", V3(0.43, 0, 0)},
      {"clr_faintblue", V3(0, 0, 0.43)}, {"clr_faintgreen", V3(0, 0.43, 0)}, {"clr_faintyellow", V3(0.43, 0.43, 0)},
      {"clr_faintcyan", V3(0, 0.43, 0.43)}, {"clr_faintmagenta", V3(0.43, 0, 0.43)}, {"clr_offwhite", V3(0.95, 0.98, 0.92)}};
  auto it = tab.find(n);
  if (it == tab.end()) {
    if (n == "clr_rnd") return false;
    c = Color(1.0, 1.0, 1.0);  // "Color not found ... so using white"
    return true;
  }
  c = Color(it->second.x, it->second.y, it->second.z);
  return true;
}

// java.util.Random (JDK 8): 48-bit LCG, setSeed scrambling, nextDouble from 26 + 27 bits
struct JRandom {
  uint64_t seed = 0;
  void set_seed(int64_t s) { seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }
  int32_t next(int bits) {
    seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(int64_t)(seed >> (48 - bits));
  }
  double next_double() { return (double)(((int64_t)next(26) << 27) + next(27)) * 0x1.0p-53; }
};
static int fastfloor(double x) { return x > 0 ? jd2i(x) : jd2i(x) - 1; }  // DistRayTracer.java:307
// myROI.calcROI variants (myTextureHandler.java:515-690) over the ascending distinct distances
static double roi(int fn, int numPts, const std::vector<double>& keys) {
  auto fix = [](double d) { if (d < 0) d *= -1; if (d > 1.0) d = 1.0 / d; return d; };
  double dist = 0;
  int i = 0, mod = -1;
  for (double k : keys) {
    switch (fn) {
      case 0: dist += k; i++; break;                                 // nearestROI
      case 2: dist += 1.0 / (mod * k); i++; break;                   // altInvLinROI
      case 3: dist += (mod * std::pow(k, ++i)); break;               // altExpROI
      case 4: dist += (mod * std::log(1 + k)); i++; break;           // altLogROI
      case 5: dist += std::pow(k, ++i); break;                       // linExpROI
      case 6: dist += std::log(1 + k); i++; break;                   // linLogROI
      case 7: dist += std::pow(k, -(++i)); break;                    // invExpROI
      case 8: dist += 1.0 / std::log(1 + k); i++; break;             // invLogROI
      default: dist += (mod * k); i++; break;                        // altLinROI (1 and unknown)
    }
    if (i >= numPts) break;
    mod *= -1;
  }
  return fn == 6 ? dist : fix(dist);  // linLogROI returns its sum unfixed
}
static const int NGHBR[27][3] = {  // DistRayTracer.nghbrHdCells (:21-25)
    {0, 0, 0},  {0, 0, 1},  {0, 0, -1},  {0, 1, 0},  {0, 1, 1},  {0, 1, -1},  {0, -1, 0},  {0, -1, 1},  {0, -1, -1},
    {1, 0, 0},  {1, 0, 1},  {1, 0, -1},  {1, 1, 0},  {1, 1, 1},  {1, 1, -1},  {1, -1, 0},  {1, -1, 1},  {1, -1, -1},
    {-1, 0, 0}, {-1, 0, 1}, {-1, 0, -1}, {-1, 1, 0}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, 0}, {-1, -1, 1}, {-1, -1, -1}};
static int32_t hash_ints(int32_t x, int32_t y, int32_t z) {  // hashInts, Java int arithmetic (wraps)
  return (int32_t)((uint32_t)x * 1572869u + (uint32_t)y * 6291469u + (uint32_t)z);
}
// myCellularTexture.getDiffTxtrColor (myTextureHandler.java:433-480)
static void cellular_color(const Shader* sh, Hit& hit, double out[3]) {
  V3 hv = sh->useFwdTrans ? hit.fwdTransHitLoc : hit.hitLoc;
  hv = V3(hv.x * sh->scale, hv.y * sh->scale, hv.z * sh->scale);
  const int idx[3] = {fastfloor(hv.x), fastfloor(hv.y), fastfloor(hv.z)};
  std::map<double, std::array<int32_t, 3>> distToPts;  // put replaces the cell of an equal distance
  JRandom rnd;
  for (int n = 0; n < 27; ++n) {
    std::array<int32_t, 3> cell = {idx[0] + NGHBR[n][0], idx[1] + NGHBR[n][1], idx[2] + NGHBR[n][2]};
    rnd.set_seed(hash_ints(cell[0], cell[1], cell[2]));
    double prob = rnd.next_double();
    auto it = sh->pdfs.lower_bound(prob);  // lowerKey(prob): greatest key < prob, else firstKey
    int numPoints = (it == sh->pdfs.begin()) ? sh->pdfs.begin()->second : std::prev(it)->second;
    for (int j = 0; j < numPoints; ++j) {
      double px = cell[0] + rnd.next_double(), py = cell[1] + rnd.next_double(), pz = cell[2] + rnd.next_double();
      double d = (sh->distFunc == 0)
                     ? std::fabs(hv.x - px) + std::fabs(hv.y - py) + std::fabs(hv.z - pz)  // _L1Dist
                     : std::sqrt(((hv.x - px) * (hv.x - px)) + ((hv.y - py) * (hv.y - py)) + ((hv.z - pz) * (hv.z - pz)));
      distToPts[d] = cell;
    }
  }
  std::vector<double> keys;
  for (auto& e : distToPts) keys.push_back(e.first);
  double dist = roi(sh->roiFunc, sh->numPtsDist, keys);
  dist = (dist < 0 ? 0 : dist > 1 ? 1 : dist);
  int brick = 2;
  if (dist < sh->mortarThresh) {
    brick = 0;
  } else {
    const std::array<int32_t, 3>& c0 = distToPts.begin()->second;
    rnd.set_seed(hash_ints(c0[0], c0[1], c0[2]));
    double res = rnd.next_double();
    brick = 2 * (1 + (fastfloor((((int)sh->colors.size() / 2) - 1) * res)));
  }
  clr_ara(sh, .65, hv, out, brick, brick + 1);
}

static void diff_txtr_color(Shader* sh, Hit& hit, double diffConst, double out[3], uint64_t* st) {
  if (sh->tex == TX_IMAGE) {  // myImageTexture.getDiffTxtrColor :105-117
    if (sh->txTop && sh->texTop) image_color(hit, *sh->texTop, out, st);
    else { out[0] = sh->diffuse.r; out[1] = sh->diffuse.g; out[2] = sh->diffuse.b; }
    out[0] *= diffConst; out[1] *= diffConst; out[2] *= diffConst;
    return;
  }
  if (sh->tex == TX_STONE) {
    cellular_color(sh, hit, out);
    if (std::fabs(diffConst - 1.0) > EPS) { out[0] *= diffConst; out[1] *= diffConst; out[2] *= diffConst; }
    return;
  }
  if (sh->tex == TX_NOISE || sh->tex == TX_MARBLE || sh->tex == TX_WOOD || sh->tex == TX_WOOD2) {
    V3 hv = sh->useFwdTrans ? hit.fwdTransHitLoc : hit.hitLoc;
    const V3& pm = sh->periodMult;
    if (sh->tex == TX_WOOD) {  // myBaseWoodTexture (myTextureHandler.java:309-331); getNoiseVal scales hitVal in place
      hv = V3(hv.x * sh->scale, hv.y * sh->scale, hv.z * sh->scale);
      double res = noise3((float)hv.x, (float)hv.y, (float)hv.z);
      double sq = std::sqrt((hv.x * hv.x) * pm.x + (hv.y * hv.y) * pm.y + (hv.z * hv.z) * pm.z) + sh->turbMult * res;
      double distVal = jf::sin(sq * mag(pm));
      distVal *= 1.1;
      distVal += .5;
      distVal = (distVal < 0 ? 0 : (distVal > 1 ? 1 : distVal));
      clr_ara(sh, distVal, hit.hitLoc, out);  // the base wood colours from the unscaled object-space hit
    } else if (sh->tex == TX_WOOD2) {  // myWoodTexture (:334-356) with getTurbVal (:225-233)
      hv = V3(hv.x * sh->scale, hv.y * sh->scale, hv.z * sh->scale);
      double res = 0, fs = 1.0, as = 1.0;
      for (int i = 0; i < sh->numOctaves; ++i) {
        res += noise3((float)(hv.x * fs), (float)(hv.y * fs), (float)(hv.z * fs)) * as;
        as *= .5;
        fs *= 1.92;
      }
      double sq = std::sqrt((hv.x * hv.x) * pm.x + (hv.y * hv.y) * pm.y + (hv.z * hv.z) * pm.z) + sh->turbMult * res;
      double distVal = (jf::sin(sq * mag(pm)));
      distVal = 1 - (distVal < 0 ? 0 : distVal);
      clr_ara(sh, distVal, hv, out);
    } else if (sh->tex == TX_NOISE) {  // myNoiseTexture :257-265
      hv = V3(hv.x * sh->scale, hv.y * sh->scale, hv.z * sh->scale);
      double res = sh->turbMult * noise3((float)hv.x, (float)hv.y, (float)hv.z);
      double val = .5 * res + .5;
      out[0] = out[1] = out[2] = val;
    } else {  // myMarbleTexture :366-377 (getAbsTurbVal scales hitVal in place :242-251)
      hv = V3(hv.x * sh->scale, hv.y * sh->scale, hv.z * sh->scale);
      double res = 0, fs = 1.0, as = 1.0;
      for (int i = 0; i < sh->numOctaves; ++i) {
        res += std::fabs(noise3((float)(hv.x * fs), (float)(hv.y * fs), (float)(hv.z * fs))) * as;
        as *= .5;
        fs *= 1.92;
      }
      double lin = (hv.x * sh->periodMult.x + hv.y * sh->periodMult.y + hv.z * sh->periodMult.z);
      double spt = lin / mag(sh->periodMult) + sh->turbMult * res;
      double distVal = .5 * jf::sin(spt) + .5;
      clr_ara(sh, distVal, hv, out);
    }
    if (std::fabs(diffConst - 1.0) > EPS) { out[0] *= diffConst; out[1] *= diffConst; out[2] *= diffConst; }
    return;
  }
  // myNonTexture :50-52
  out[0] = sh->diffuse.r * diffConst; out[1] = sh->diffuse.g * diffConst; out[2] = sh->diffuse.b * diffConst;
}

// calcShadowColor (myObjShader.java:98-153)
static void shadow_color(Scene* s, Shader* sh, Hit& hit, const double tex[3], double out[3], uint64_t* st) {
  double r = 0, g = 0, b = 0;
  V3 hitLoc = hit.fwdTransHitLoc;
  for (Light* L : s->lightList) {
    RKey k = hit.transRay.key;
    V3 lo = (L->ltype == LT_DISK) ? L->disk_pos(k, 0) : L->origin;
    V3 ln = xpt(L->ctm->g, lo);
    ln = V3(ln.x - hitLoc.x, ln.y - hitLoc.y, ln.z - hitLoc.z);
    normalize_ip(ln);
    Ray sr(hitLoc, ln, hit.transRay.gen + 1);
    sr.key = k;
    sr.key.time_site = SITE_SHADOW_TIME + L->index;
    // light.intersectCheck (myLight.java:33-41, spot :159-163)
    V3 lo2 = (L->ltype == LT_DISK) ? L->disk_pos(k, 2) : L->origin;
    double t = dist(sr.origin, lo2);
    double ltMult = 1;
    if (st) st[ST_LIGHT]++;
    if (L->ltype == LT_SPOT) {
      double angle = jf::acos(-1 * dot(sr.direction, L->orientation));
      ltMult = L->angle_prob(angle);
    }
    if (ltMult == 0) continue;
    if (st) st[ST_SHADOW]++;
    int blocked = calc_shadow(s, sr, t, st);
    if (blocked == 0) {
      normalize_ip(sr.direction);
      double ld = dot(sr.direction, hit.objNorm) * ltMult;
      if (ld > EPS) {
        r += tex[0] * L->lightColor.r * ld;
        g += tex[1] * L->lightColor.g * ld;
        b += tex[2] * L->lightColor.b * ld;
      }
      if (sh->phongExp == 0) continue;
      V3 hN(sr.direction.x - hit.fwdTransRayDir.x, sr.direction.y - hit.fwdTransRayDir.y, sr.direction.z - hit.fwdTransRayDir.z);
      normalize_ip(hN);
      double hd = dot(hN, hit.objNorm) * ltMult;
      if (hd > EPS) {
        double ph = std::pow(hd * hd, sh->phongExp);
        r += sh->specular.r * L->lightColor.r * ph;
        g += sh->specular.g * L->lightColor.g * ph;
        b += sh->specular.b * L->lightColor.b * ph;
      }
    }
  }
  out[0] = r; out[1] = g; out[2] = b;
}

static V3 refl_dir(const V3& eye, const V3& n) {  // compReflDir :89-96
  double dp = 2 * dot(eye, n);
  V3 tv(n.x * dp, n.y * dp, n.z * dp);
  V3 r = vsub(tv, eye);
  normalize_ip(r);
  return r;
}
static double angle_between(const V3& v1, const V3& v2) {  // DistRayTracer.java:445-452
  double m1 = mag(v1), m2 = mag(v2), dp = dot(v1, v2), ca = dp / (m1 * m2);
  return jf::acos(ca);
}
static double fres_perp(double n1, double n2, double ci, double ct) { double a = n1 * ci, b = n2 * ct, nd = (a - b) / (a + b); return nd * nd; }
static double fres_plel(double n1, double n2, double ci, double ct) { double a = n1 * ct, b = n2 * ci, nd = (a - b) / (a + b); return nd * nd; }

// Fresnel split shared by calcTransClr (:157-276), calcTransRay (:297-397) and the
// simple shader (:503-631). `simple` selects mySimpleReflObjShdr's index choice.
struct TransSplit {
  V3 N, back, reflDir, refrDir;
  double n = 1, n1 = 0, n2 = 0, cos1 = 0, cos2 = 0, tr = 0, omtr = 1, refractNormMult = 1;
  bool TIR = false;
};
static TransSplit trans_split(const Shader* sh, const Hit& hit, bool simple) {
  TransSplit S;
  S.back = V3(hit.fwdTransRayDir.x * -1, hit.fwdTransRayDir.y * -1, hit.fwdTransRayDir.z * -1);
  S.N = hit.objNorm;
  double exitT = 1;
  double cos1 = dot(S.back, S.N);
  if (cos1 < EPS) { S.refractNormMult = -1.0; S.N = V3(S.N.x * -1, S.N.y * -1, S.N.z * -1); }
  cos1 = dot(S.back, S.N);
  double thetaI = angle_between(S.back, S.N);
  double idx = simple ? sh->currPerm : sh->KTrans;
  if (simple) S.reflDir = refl_dir(S.back, S.N);
  if (S.refractNormMult < 0) {
    double thetaCrit = jf::asin(exitT / idx);
    if (thetaI < thetaCrit) {
      S.n1 = idx; S.n2 = exitT; S.n = (S.n1 / S.n2);
      double c2 = 1.0 - (S.n * S.n) * (1.0 - (cos1 * cos1));
      S.cos2 = std::sqrt(c2);
    } else {
      S.tr = 1; S.omtr = 1 - S.tr; S.TIR = true; S.cos2 = 0;
    }
  } else {
    S.n1 = simple ? hit.transRay.kt[1] : hit.transRay.kt[0];
    S.n2 = idx;
    S.n = (S.n1 / S.n2);
    double c2 = 1.0 - (S.n * S.n) * (1.0 - (cos1 * cos1));
    S.cos2 = std::sqrt(c2);
  }
  if (!S.TIR) {
    double sa = jf::sin(jf::acos(cos1)), rct = std::sqrt(1.0 - ((S.n1 / S.n2) * sa * sa));
    double rp = fres_perp(S.n1, S.n2, cos1, rct), rl = fres_plel(S.n1, S.n2, cos1, rct);
    S.tr = (rp + rl) / 2.0;
    S.omtr = 1 - S.tr;
  }
  S.cos1 = cos1;
  V3 u(S.back.x * (S.n * -1), S.back.y * (S.n * -1), S.back.z * (S.n * -1));
  double k = (S.n * cos1) - S.cos2;
  V3 nv(S.N.x * k, S.N.y * k, S.N.z * k);
  S.refrDir = V3(u.x + nv.x, u.y + nv.y, u.z + nv.z);
  normalize_ip(S.refrDir);
  return S;
}

static Color shade(Scene* s, Hit& hit, uint64_t* st) {
  Shader* sh = hit.shdr;
  double r = sh->ambient.r, g = sh->ambient.g, b = sh->ambient.b;
  const uint32_t node = hit.transRay.key.node;
  if (!sh->simple) {  // myObjShader.getColorAtPos :409-438
    if ((sh->KRefl == 0.0) && sh->usePhotonMap) {
      double ir[3];
      s->photonTree.irradiance(hit.fwdTransHitLoc, ir, st);
      if (sh->isCausticPhtn) { r += ir[0]; g += ir[1]; b += ir[2]; }
      else { r += sh->diffuse.r * ir[0]; g += sh->diffuse.g * ir[1]; b += sh->diffuse.b * ir[2]; }
    }
  }
  double tex[3], sres[3];
  diff_txtr_color(sh, hit, sh->simple ? 1.0 : sh->diffConst, tex, st);
  shadow_color(s, sh, hit, tex, sres, st);
  r += sres[0]; g += sres[1]; b += sres[2];
  if ((hit.transRay.gen < s->numRays - 2) && sh->hasCaustic) {
    double res[3] = {0, 0, 0};
    V3 hitLoc = hit.fwdTransHitLoc;
    if (!sh->simple && ((sh->KTrans > 0) || (sh->currPerm > 0.0))) {  // calcTransClr
      TransSplit S = trans_split(sh, hit, false);
      if (S.omtr > EPS) {
        Ray rr(hitLoc, S.refrDir, hit.transRay.gen + 1);
        rr.kt[0] = sh->KTrans; rr.kt[1] = sh->currPerm; rr.kt[2] = sh->curPermClr.r; rr.kt[3] = sh->curPermClr.g; rr.kt[4] = sh->curPermClr.b;
        rr.key = hit.transRay.key; rr.key.node = node * 2; rr.key.time_site = SITE_TIME;
        if (st) st[ST_REFR]++;
        Color c = reflect_ray(s, rr, st);
        res[0] += (S.omtr) * sh->curPermClr.r * (c.r);
        res[1] += (S.omtr) * sh->curPermClr.g * (c.g);
        res[2] += (S.omtr) * sh->curPermClr.b * (c.b);
      }
      if (S.tr > EPS) {
        V3 rd = refl_dir(S.back, S.N);
        rd = V3(rd.x * S.refractNormMult, rd.y * S.refractNormMult, rd.z * S.refractNormMult);
        Ray rr(hitLoc, rd, hit.transRay.gen + 1);
        rr.kt[0] = sh->KTrans; rr.kt[1] = sh->currPerm; rr.kt[2] = sh->curPermClr.r; rr.kt[3] = sh->curPermClr.g; rr.kt[4] = sh->curPermClr.b;
        rr.key = hit.transRay.key; rr.key.node = node * 2 + 1; rr.key.time_site = SITE_TIME;
        if (st) st[ST_REFL]++;
        Color c = reflect_ray(s, rr, st);
        res[0] += (S.tr) * sh->curPermClr.r * (c.r);
        res[1] += (S.tr) * sh->curPermClr.g * (c.g);
        res[2] += (S.tr) * sh->curPermClr.b * (c.b);
      }
    } else if (sh->simple && sh->KTrans > 0) {  // calcSimpleTransClr :503-631
      TransSplit S = trans_split(sh, hit, true);
      if (S.omtr > 0) {
        Ray rr(hitLoc, S.refrDir, hit.transRay.gen + 1);
        rr.kt[0] = sh->KTrans; rr.kt[1] = sh->currPerm; rr.kt[2] = sh->curPermClr.r; rr.kt[3] = sh->curPermClr.g; rr.kt[4] = sh->curPermClr.b;
        rr.key = hit.transRay.key; rr.key.node = node * 2; rr.key.time_site = SITE_TIME;
        if (st) st[ST_REFR]++;
        Color c = reflect_ray(s, rr, st);
        double pm = S.omtr * sh->KTrans;
        res[0] += pm * (c.r); res[1] += pm * (c.g); res[2] += pm * (c.b);
      }
      if (S.tr > 0) {
        V3 rd(S.reflDir.x * S.refractNormMult, S.reflDir.y * S.refractNormMult, S.reflDir.z * S.refractNormMult);
        Ray rr(hitLoc, rd, hit.transRay.gen + 1);
        rr.key = hit.transRay.key; rr.key.node = node * 2 + 1; rr.key.time_site = SITE_TIME;
        if (st) st[ST_REFL]++;
        Color c = reflect_ray(s, rr, st);
        double pm = S.tr * sh->KRefl;
        res[0] += pm * (c.r); res[1] += pm * (c.g); res[2] += pm * (c.b);
      }
    } else if (sh->KRefl > 0.0) {  // calcReflClr :278-294
      V3 back(hit.fwdTransRayDir.x * -1, hit.fwdTransRayDir.y * -1, hit.fwdTransRayDir.z * -1);
      V3 rd = refl_dir(back, hit.objNorm);
      if (dot(rd, hit.objNorm) >= 0) {
        Ray rr(hitLoc, rd, hit.transRay.gen + 1);
        rr.key = hit.transRay.key; rr.key.node = node * 2; rr.key.time_site = SITE_TIME;
        if (st) st[ST_REFL]++;
        Color c = reflect_ray(s, rr, st);
        res[0] += (sh->KReflClr.r * c.r);
        res[1] += (sh->KReflClr.g * c.g);
        res[2] += (sh->KReflClr.b * c.b);
      }
    }
    r += res[0]; g += res[1]; b += res[2];
  }
  return Color(r, g, b);
}

// ---------------------------------------------------------------------------
// photon pre-pass (myScene.java:952-1099), keyed: pixel field = photon index,
// sample field = light index, node field = bounce.
static double pdraw(Scene* s, uint64_t seed, uint64_t i, uint32_t light, uint32_t bounce, uint32_t site, uint32_t k, double a, double b) {
  return rng_range(rng_bits(seed, i, light, bounce, site, k), a, b);
}
static Ray photon_ray(Scene* s, Light* L, uint64_t seed, uint64_t i) {  // genRndPhtnRay
  uint32_t k = 0;
  V3 dir;
  uint32_t li = (uint32_t)L->index;
  if (L->ltype == LT_POINT) {  // getRandDir :59-74
    double x, y, z, sq;
    do {
      x = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      y = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      z = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, -1.0, 1.0);
      sq = (x * x) + (y * y) + (z * z);
    } while ((sq > 1.0) || (sq < EPS));
    double m = std::sqrt(sq);
    dir = V3(x / m, y / m, z / m);
    return Ray(xpt(L->ctm->g, L->origin), dir, 0);
  }
  if (L->ltype == LT_SPOT) {  // :165-185
    double checkProb = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, 1), angle, prob;
    do {
      angle = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, L->outerRad);
      prob = L->angle_prob(angle);
    } while (prob > checkProb);
    V3 t = rot_around_axis(L->orientation, L->oPhAxis, angle);
    normalize_ip(t);
    t = rot_around_axis(t, L->orientation, pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, TWO_PI_F));
    return Ray(xpt(L->ctm->g, L->origin), t, 0);
  }
  // disk :229-242 (getAngleProb(angle, 0, PI, PI))
  double angle, prob;
  do {
    angle = pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, M_PI);
    prob = (angle < 0) ? 1 : (angle > M_PI) ? 0 : (M_PI - angle) / M_PI;
  } while (prob > pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, 1));
  V3 d = rot_around_axis(L->orientation, L->surfTangent, angle);
  normalize_ip(d);
  d = rot_around_axis(d, L->orientation, pdraw(s, seed, i, li, 0, SITE_PH_DIR, k++, 0, TWO_PI_F));
  RKey kk;
  kk.seed = seed; kk.pixel = i; kk.sample = li; kk.node = 0;
  // disk position draws use the photon sub-key (site SITE_DISK + light)
  V3 loc = L->disk_pos(kk, 0);
  return Ray(xpt(L->ctm->g, loc), d, 0);
}
static Ray caustic_ray(Scene* s, Hit& hit, double pwr[3], bool& ok) {  // findCausticRayHit :461-478
  ok = false;
  Shader* sh = hit.shdr;
  Ray res;
  if ((hit.transRay.gen < s->numPhotonRays) && sh->hasCaustic) {
    double pm[3] = {1.0, 1.0, 1.0};
    if ((sh->KTrans > 0.0) || (sh->currPerm > 0.0)) {
      pm[0] = sh->phtnPermClr.x; pm[1] = sh->phtnPermClr.y; pm[2] = sh->phtnPermClr.z;
      TransSplit S = trans_split(sh, hit, false);
      if (S.omtr > EPS) res = Ray(hit.fwdTransHitLoc, S.refrDir, hit.transRay.gen + 1);
      else {
        V3 rd = refl_dir(S.back, S.N);
        rd = V3(rd.x * S.refractNormMult, rd.y * S.refractNormMult, rd.z * S.refractNormMult);
        res = Ray(hit.fwdTransHitLoc, rd, hit.transRay.gen + 1);
      }
      res.kt[0] = sh->KTrans; res.kt[1] = sh->currPerm; res.kt[2] = sh->curPermClr.r; res.kt[3] = sh->curPermClr.g; res.kt[4] = sh->curPermClr.b;
      ok = true;
    } else if (sh->KRefl > 0.0) {
      pm[0] = pm[1] = pm[2] = sh->KRefl;
      V3 back(hit.fwdTransRayDir.x * -1, hit.fwdTransRayDir.y * -1, hit.fwdTransRayDir.z * -1);
      res = Ray(hit.fwdTransHitLoc, refl_dir(back, hit.objNorm), hit.transRay.gen + 1);
      ok = true;
    }
    for (int i = 0; i < 3; ++i) hit.phtnPwr[i] = pwr[i] * pm[i];
  }
  return res;
}
static void send_photons(Scene* s, uint64_t seed) {
  KDTree& T = s->photonTree;
  T.photons.clear();
  bool caustic = s->isCausticPhtn;
  double pwrMult = (caustic ? s->causticsLightPwrMult : s->diffuseLightPwrMult) / T.num_Cast;
  for (Light* L : s->lightList) {
    uint32_t li = (uint32_t)L->index;
    for (int i = 0; i < T.num_Cast; ++i) {
      double ppwr[3] = {L->lightColor.r * pwrMult, L->lightColor.g * pwrMult, L->lightColor.b * pwrMult};
      Ray pr = photon_ray(s, L, seed, (uint64_t)i);
      pr.key.seed = seed; pr.key.pixel = (uint64_t)i; pr.key.sample = li; pr.key.node = 0; pr.key.time_site = SITE_PH_TIME;
      Hit h = closest_hit(s, pr, nullptr);
      if (caustic) {  // sendCausticPhotons :952-998
        if (!h.isHit || !h.shdr->hasCaustic) continue;
        for (int c = 0; c < 3; ++c) h.phtnPwr[c] = ppwr[c];
        bool ok;
        int gen = 0;
        do {
          double cur[3] = {h.phtnPwr[0], h.phtnPwr[1], h.phtnPwr[2]};
          Ray rr = caustic_ray(s, h, cur, ok);
          if (ok) {
            double tp[3] = {h.phtnPwr[0], h.phtnPwr[1], h.phtnPwr[2]};
            gen = rr.gen;
            rr.key = pr.key; rr.key.node = (uint32_t)gen;
            h = closest_hit(s, rr, nullptr);
            for (int c = 0; c < 3; ++c) h.phtnPwr[c] = tp[c];
          } else h.isHit = false;
        } while (h.isHit && h.shdr->hasCaustic && gen <= s->numPhotonRays);
        if (!h.isHit || gen > s->numPhotonRays) continue;
        Photon p;
        p.pwr[0] = h.phtnPwr[0]; p.pwr[1] = h.phtnPwr[1]; p.pwr[2] = h.phtnPwr[2];
        p.pos[0] = h.fwdTransHitLoc.x; p.pos[1] = h.fwdTransHitLoc.y; p.pos[2] = h.fwdTransHitLoc.z; p.pos[3] = 0;
        T.photons.push_back(p);
      } else {  // sendDiffusePhotons :1000-1091
        if (!h.isHit) continue;
        for (int c = 0; c < 3; ++c) h.phtnPwr[c] = ppwr[c];
        bool done = false, firstDiff = true;
        uint32_t bounce = 0;
        do {
          bounce++;
          if (h.shdr->KRefl == 0) {
            double prob = 0;
            uint32_t k = 0;
            if (!firstDiff) {
              Photon p;
              p.pwr[0] = h.phtnPwr[0]; p.pwr[1] = h.phtnPwr[1]; p.pwr[2] = h.phtnPwr[2];
              p.pos[0] = h.fwdTransHitLoc.x; p.pos[1] = h.fwdTransHitLoc.y; p.pos[2] = h.fwdTransHitLoc.z; p.pos[3] = 0;
              T.photons.push_back(p);
              prob = pdraw(s, seed, (uint64_t)i, li, bounce, SITE_PH_BOUNCE, k++, 0, 1.0);
            }
            firstDiff = false;
            if (prob < h.shdr->avgDiffClr) {
              V3 hitLoc = h.fwdTransHitLoc;
              double x = 0, y = 0, z = 0, sq;
              do {
                x = pdraw(s, seed, (uint64_t)i, li, bounce, SITE_PH_BOUNCE, k++, -1.0, 1.0);
                y = pdraw(s, seed, (uint64_t)i, li, bounce, SITE_PH_BOUNCE, k++, -1.0, 1.0);
                sq = (x * x) + (y * y);
              } while ((sq >= 1.0) || (sq < EPS));
              z = std::sqrt(1 - (sq));
              V3 n = h.objNorm;
              double nx = n.x * n.x, ny = n.y * n.y, nz = n.z * n.z;
              V3 tv = ((nx > ny) && (nx > nz)) ? V3(0, 0, 1) : V3(1, 0, 0);
              V3 p_ = cross(n, tv), q_ = cross(p_, n);
              n = V3(n.x * z, n.y * z, n.z * z);
              p_ = V3(p_.x * x, p_.y * x, p_.z * x);
              q_ = V3(q_.x * y, q_.y * y, q_.z * y);
              V3 bd(n.x + p_.x + q_.x, n.y + p_.y + q_.y, n.z + p_.z + q_.z);
              normalize_ip(bd);
              double tp[3] = {h.phtnPwr[0] * h.shdr->phtnDiffScl.x, h.phtnPwr[1] * h.shdr->phtnDiffScl.y, h.phtnPwr[2] * h.shdr->phtnDiffScl.z};
              Ray rr(hitLoc, bd, h.transRay.gen + 1);
              rr.key = pr.key; rr.key.node = bounce;
              h = closest_hit(s, rr, nullptr);
              for (int c = 0; c < 3; ++c) h.phtnPwr[c] = tp[c];
            } else done = true;
          } else {
            double cur[3] = {h.phtnPwr[0], h.phtnPwr[1], h.phtnPwr[2]};
            bool ok;
            Ray rr = caustic_ray(s, h, cur, ok);
            if (ok) {
              double tp[3] = {h.phtnPwr[0], h.phtnPwr[1], h.phtnPwr[2]};
              rr.key = pr.key; rr.key.node = bounce;
              h = closest_hit(s, rr, nullptr);
              for (int c = 0; c < 3; ++c) h.phtnPwr[c] = tp[c];
            } else h.isHit = false;
          }
        } while (h.isHit && !done && h.transRay.gen <= s->numPhotonRays);
      }
    }
  }
  T.build_all();
  s->photonsBuilt = true;
}

// ---------------------------------------------------------------------------
// .cli loader (myRTFileReader.java:15-349), subset used by the hot path + builder state (myScene.java)
struct Loader {
  Scene* s;
  std::string dir;
  std::vector<M4> stack{M4()};
  // current material state (myScene.java:144-145, setSurface :817-850)
  Color cDiff, cAmb, cSpec, permClr, kReflClr;
  double phong = 0, kRefl = 0, kTrans = 0, rfrIdx = 0;
  bool simpleRefr = false, txTop = false, txBtm = false;
  int txtrType = 0;
  std::string texTopName;
  // proc texture state (myScene.java:117-139)
  double noiseScale = 1, turbMult = 1, colorScale = 10, colorMult = .2;
  int numOctaves = 8;
  V3 pdMult{10, 10, 10};
  bool rndColors = false, useFwdTrans = false, useCustClrs = false;
  std::vector<Color> noiseColors{Color(.7, .7, .7), Color(.2, .2, .2)};
  int numPtsDist = 2, distFunc = 1, roiFunc = 1;
  double avgNumPerCell = 1.0, mortarThresh = 0.05;
  bool inTmpList = false;
  std::vector<GeomBase*> tmpList;
  std::map<std::string, GeomBase*> named;  // namedObjs (myScene.java:378-387)
  int curNumRaysPerPxl = 0;
  std::string err;
  int ignored = 0;  // unknown commands skipped (myRTFileReader.java:343-345)

  std::shared_ptr<CTM> cur_ctm() { return std::make_shared<CTM>(build_ctm(stack.back())); }
  void set_surface(Color d, Color a, Color sp, double ph, double kr) {
    txtrType = 0;
    cDiff = d; cAmb = a; cSpec = sp; phong = ph;
    kRefl = kr; kReflClr = Color(kr, kr, kr);
    rfrIdx = 0; permClr = Color(0, 0, 0);
    kTrans = 0;
  }
  Shader* cur_shader() {  // getCurShader (myScene.java:524-528) + setCurrColors (myObjShader.java:51-75)
    Shader* sh = new Shader();
    s->shaders.emplace_back(sh);
    sh->simple = simpleRefr;
    sh->diffuse = cDiff;
    auto avg = [](const Color& c) { return (1.0 / 3.0) * (c.r + c.g + c.b); };
    sh->avgDiffClr = avg(cDiff);
    if (sh->avgDiffClr != 0) sh->phtnDiffScl = V3(cDiff.r / sh->avgDiffClr, cDiff.g / sh->avgDiffClr, cDiff.b / sh->avgDiffClr);
    sh->ambient = cAmb;
    sh->specular = cSpec;
    sh->avgSpecClr = avg(cSpec);
    sh->KRefl = kRefl;
    sh->KReflClr = kReflClr;
    sh->KTrans = kTrans;
    sh->curPermClr = permClr;
    sh->avgPermClr = avg(permClr);
    if (sh->avgPermClr != 0) sh->phtnPermClr = V3(permClr.r / sh->avgPermClr, permClr.g / sh->avgPermClr, permClr.b / sh->avgPermClr);
    sh->currPerm = rfrIdx;
    sh->hasCaustic = ((kRefl > 0.0) || (rfrIdx > 0.0) || (kTrans > 0.0));
    sh->usePhotonMap = s->usePhotonMap;
    sh->isCausticPhtn = s->isCausticPhtn;
    sh->diffConst = 1 - rfrIdx;
    sh->phongExp = phong;
    sh->tex = (txtrType >= 1 && txtrType <= 6) ? txtrType : TX_NONE;
    if (txtrType == 1) {
      sh->txTop = txTop;
      if (txTop) {
        auto it = s->textures->find(texTopName);
        if (it == s->textures->end()) { err = "texture not registered: " + texTopName; sh->txTop = false; }
        else sh->texTop = &it->second;
      }
    }
    if (txtrType == 5) {  // myCellularTexture ctor (myTextureHandler.java:390-425)
      sh->numPtsDist = numPtsDist; sh->distFunc = distFunc; sh->roiFunc = roiFunc; sh->mortarThresh = mortarThresh;
      double lastDist = 1.0 / std::pow(M_E, avgNumPerCell), cumProb = lastDist;
      for (int i = 1; i < 15; ++i) {
        lastDist *= (avgNumPerCell / (1.0 * i));
        cumProb += lastDist;
        sh->pdfs[cumProb] = i;
      }
    }
    if (txtrType == 2 || txtrType == 3 || txtrType == 4 || txtrType == 5 || txtrType == 6) {
      while (noiseColors.size() < 2) noiseColors.push_back(Color(1, 1, 1));  // (Java would throw at render)
      sh->scale = noiseScale; sh->numOctaves = numOctaves; sh->turbMult = turbMult; sh->periodMult = pdMult;
      sh->colorScale = colorScale; sh->colorMult = colorMult; sh->rndColors = rndColors; sh->useFwdTrans = useFwdTrans;
      sh->colors = noiseColors;
    }
    return sh;
  }
  void add_object(GeomBase* o) {  // addObjectToScene (myScene.java:558-565)
    if (inTmpList) { tmpList.push_back(o); return; }
    if (o->isLight) s->lightList.push_back(static_cast<Light*>(o));
    else s->objList.push_back(o);
  }
  void reset_dflt_txtr() {  // resetDfltTxtrVals (myScene.java:579-586)
    txtrType = 0; numOctaves = 4; rndColors = false; useCustClrs = false; useFwdTrans = false;
    noiseScale = 1.0; turbMult = 1.0; colorScale = 5.0; colorMult = .1;
    pdMult = V3(1.0, 1.0, 1.0);
    noiseColors = {Color(0.05, 0.05, 0.05), Color(1.0, 1.0, 1.0)};
    numPtsDist = 2; distFunc = 1; roiFunc = 1; avgNumPerCell = 1.0; mortarThresh = 0.05;
  }
  bool read_worley(const std::vector<std::string>& v) {  // readProcTxtrWorleyVals (myScene.java:675-708)
    try {
      size_t k = 1;
      noiseScale = std::stod(v.at(k++));
      distFunc = std::stoi(v.at(k++));
      roiFunc = std::stoi(v.at(k++));
      numPtsDist = std::stoi(v.at(k++));
      avgNumPerCell = std::stod(v.at(k++));
      mortarThresh = std::stod(v.at(k++));
      useFwdTrans = (std::stod(v.at(k++)) == 1.0);
      if (v.size() >= k + 2) {
        colorScale = std::stod(v.at(k)); colorMult = std::stod(v.at(k + 1)); rndColors = true;
      } else {
        rndColors = false; colorScale = 25.0; colorMult = .1;
      }
      return false;
    } catch (...) {
      return true;
    }
  }
  bool read_perlin(const std::vector<std::string>& v) {  // readProcTxtrPerlinVals (myScene.java:642-672)
    try {
      if (v.size() < 11) return true;
      noiseScale = std::stod(v.at(1));
      numOctaves = std::stoi(v.at(2));
      turbMult = std::stod(v.at(3));
      pdMult = V3(std::stod(v.at(4)), std::stod(v.at(5)), std::stod(v.at(6)));
      V3 py(std::stod(v.at(7)), std::stod(v.at(8)), std::stod(v.at(9)));
      if (sqmag(py) > 0) {
        py = V3(py.x * (TWO_PI_F - 1.0), py.y * (TWO_PI_F - 1.0), py.z * (TWO_PI_F - 1.0));
        py = V3(py.x + 1.0, py.y + 1.0, py.z + 1.0);
        pdMult = V3(pdMult.x * py.x, pdMult.y * py.y, pdMult.z * py.z);
      }
      useFwdTrans = (std::stod(v.at(10)) == 1.0);
      if (v.size() >= 13) {
        colorScale = std::stod(v.at(11));
        colorMult = std::stod(v.at(12));
        rndColors = true;
      } else {
        rndColors = false; colorScale = 25.0; colorMult = .1;
      }
      return false;
    } catch (...) {
      return true;
    }
  }
  double num(const std::vector<std::string>& t, size_t i) { return std::stod(t.at(i)); }
  // gtTranslate / gtScale / gtRotate (myScene.java:1256-1318)
  void translate(double x, double y, double z) {
    M4 T; T.m[0][3] = x; T.m[1][3] = y; T.m[2][3] = z;
    stack.back() = mmul(stack.back(), T);
  }
  void scale(double x, double y, double z) {
    M4 S; S.m[0][0] = x; S.m[1][1] = y; S.m[2][2] = z;
    stack.back() = mmul(stack.back(), S);
  }
  void rotate(double ang, double ax, double ay, double az) {
    double ar = (double)(ang * M_PI) / 180.0;
    V3 av = normalized(V3(ax, ay, az));
    V3 nv = (ax == 0) ? V3(1, 0, 0) : V3(0, 1, 0);
    V3 bv = normalized(cross(av, nv));
    V3 cv = normalized(cross(av, bv));
    M4 R1, R2;
    R1.m[0][0] = av.x; R1.m[0][1] = av.y; R1.m[0][2] = av.z;
    R1.m[1][0] = bv.x; R1.m[1][1] = bv.y; R1.m[1][2] = bv.z;
    R1.m[2][0] = cv.x; R1.m[2][1] = cv.y; R1.m[2][2] = cv.z;
    M4 R1T = transpose(R1);
    R2.m[1][1] = jf::cos(ar); R2.m[1][2] = -jf::sin(ar); R2.m[2][1] = jf::sin(ar); R2.m[2][2] = jf::cos(ar);
    M4 tmp = mmul(R2, R1);
    stack.back() = mmul(stack.back(), mmul(R1T, tmp));
  }
  void push() { stack.push_back(stack.back()); }
  void pop() { if (stack.size() > 1) stack.pop_back(); }
  // addInstance (myScene.java:389-395) + myInstance ctor (mySceneObject.java:98-110)
  bool add_instance(const std::string& name, bool addShdr) {
    auto it = named.find(name);
    if (it == named.end()) { err = "unknown named object: " + name; return false; }
    Instance* in = s->make<Instance>();
    in->obj = it->second;
    // myGeomBase ctor: origin (0,0,0) through the stack top; then CTMara = buildCTMara(scene,
    // obj.glbl) = obj.glbl x stack top (DistRayTracer.java:401)
    in->trans_origin = xpt(stack.back(), V3(0, 0, 0));
    in->ctm = std::make_shared<CTM>(build_ctm(mmul(in->obj->ctm->g, stack.back())));
    in->minVals = in->getMinVec();
    in->maxVals = in->getMaxVec();
    make_bbox(s, in);
    in->key = in->obj->key;  // RNG prim key: the named object's (instances are not primitives)
    if (addShdr) { in->useShader = true; in->shdr = cur_shader(); }
    add_object(in);
    return true;
  }
  // setSierpShdr (myScene.java:328-337), float arithmetic as in the reference
  void sierp_shader(int level, int maxLevel) {
    float bVal = 1.0f - std::min(1.0f, (1.5f * level / maxLevel)), rVal = 1.0f - bVal,
          tmp = std::min((1.2f * (level - (maxLevel / 2))) / (1.0f * maxLevel), 1.0f), gVal = (tmp * tmp);
    Color cd(std::min(1.0f, rVal + .5f), std::min(1.0f, gVal + .5f), std::min(1.0f, bVal + .5f));
    txTop = false; txBtm = false;
    set_surface(cd, Color(0, 0, 0), Color(0, 0, 0), 0, 0);
  }
  void sierp_shift(float newTrans) { rotate(120, 1, 0, 0); translate(0, newTrans, 0); rotate(-120, 1, 0, 0); }
  // buildSierpSubTri (myScene.java:339-380)
  bool sierp_sub(float dim, float scVal, const std::string& name, int level, int maxLevel, bool addShader) {
    if (level >= maxLevel) return true;
    float newDim = scVal * dim;
    push();
    translate(0, .1f * dim, 0);
    rotate(70, 0, 1, 0);
    if (addShader) sierp_shader(level, maxLevel);
    if (!add_instance(name, addShader)) return false;
    pop();
    const float sqrt66 = (float)std::sqrt(6.0f) / 6.0f;  // DistRayTracer.java:38
    float newTrans = sqrt66 * dim;
    for (int k = 0; k < 4; ++k) {  // up, front, left, right
      push();
      if (k == 0) translate(0, newTrans, 0);
      else if (k == 1) sierp_shift(newTrans);
      else if (k == 2) { rotate(120, 0, 1, 0); sierp_shift(newTrans); rotate(-120, 0, 1, 0); }
      else { rotate(-120, 0, 1, 0); sierp_shift(newTrans); rotate(120, 0, 1, 0); }
      scale(scVal, scVal, scVal);
      if (!sierp_sub(newDim, scVal, name, level + 1, maxLevel, addShader)) return false;
      pop();
    }
    return true;
  }
  void end_tmp_list(bool bvh) {  // endTmpObjList (myScene.java:305-324)
    inTmpList = false;
    if (!bvh) {
      GeomList* gl = s->make<GeomList>();
      gl->ctm = cur_ctm();
      make_bbox(s, gl);
      for (GeomBase* o : tmpList) gl->add_obj(o);
      add_object(gl);
    } else {
      BVH* root = new_bvh(s, cur_ctm());
      OList l[3];
      build_sorted(tmpList, -1, l);
      add_obj_list(s, root, l, 0, (int)l[0].size() - 1);
      add_object(root);
    }
    tmpList.clear();
  }

  bool read_file(const std::string& fname, bool isMain) {
    std::ifstream f(dir + "/" + fname);
    if (!f) { err = "cannot open " + dir + "/" + fname; return false; }
    std::string line;
    Planar* poly = nullptr;
    std::string vertType = "triangle";
    int vc = 0;
    while (std::getline(f, line)) {
      std::vector<std::string> t;
      {
        std::string cur;
        for (char ch : line) {  // splitTokens(line, " ") -- tabs/CR as whitespace too
          if (ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n') { if (!cur.empty()) { t.push_back(cur); cur.clear(); } }
          else cur.push_back(ch);
        }
        if (!cur.empty()) t.push_back(cur);
      }
      if (t.empty() || t[0][0] == '#') continue;
      const std::string& c = t[0];
      try {
        if (c == "fov") {
          if (!isMain) continue;
          s->numRaysPerPixel = (curNumRaysPerPxl != 0) ? curNumRaysPerPxl : 1;
          s->fov = num(t, 1);
          s->camType = 0;
        } else if (c == "fisheye" || c == "fishEye") {  // myRTFileReader.java:66-74
          if (!isMain) continue;
          s->numRaysPerPixel = (curNumRaysPerPxl != 0) ? curNumRaysPerPxl : 1;
          s->camType = 1;
          s->fishEye = num(t, 1);
        } else if (c == "ortho" || c == "orthographic") {  // myRTFileReader.java:75-83
          if (!isMain) continue;
          s->numRaysPerPixel = (curNumRaysPerPxl != 0) ? curNumRaysPerPxl : 1;
          s->camType = 2;
          s->orthoW = num(t, 1);
          s->orthoH = num(t, 2);
        } else if (c == "lens") {
          s->hasDOF = true; s->lensRadius = num(t, 1); s->lensFocal = num(t, 2);
        } else if (c == "write") {
          break;  // render happens at write; rest of file ignored by the oracle
        } else if (c == "read") {
          if (!read_file(t.at(1), false)) return false;
        } else if (c == "rays_per_pixel") {
          curNumRaysPerPxl = std::stoi(t.at(1));
          s->numRaysPerPixel = curNumRaysPerPxl;
        } else if (c == "antialias") {
          curNumRaysPerPxl = std::stoi(t.at(1)) * std::stoi(t.at(2));
          s->numRaysPerPixel = curNumRaysPerPxl;
        } else if (c == "background") {
          if (t.at(1) == "texture") {
            auto it = s->textures->find(t.at(2));
            if (it == s->textures->end()) { err = "texture not registered: " + t.at(2); return false; }
            s->bkgTex = &it->second;
            s->txtrdBkg = true;
            Sphere* sd = s->make<Sphere>();
            sd->ctm = cur_ctm();
            sd->radX = sd->radY = sd->radZ = num(t, 3);
            sd->origin = V3(num(t, 4), num(t, 5), num(t, 6));
            s->skyDome = sd;
          } else {
            s->backgroundColor = Color(num(t, 1), num(t, 2), num(t, 3));
            txtrType = 0;
          }
        } else if (c == "point_light" || c == "spotlight" || c == "disk_light") {
          Light* L = s->make<Light>();
          L->isLight = true;
          L->ctm = cur_ctm();
          L->index = (int)s->lightList.size();
          if (c == "point_light") {  // addMyPointLight (myScene.java:413-419)
            L->ltype = LT_POINT;
            L->origin = V3(num(t, 1), num(t, 2), num(t, 3));
            L->lightColor = Color(num(t, 4), num(t, 5), num(t, 6));
          } else if (c == "spotlight") {  // :422-432, myLight.java:150-157
            L->ltype = LT_SPOT;
            L->origin = V3(num(t, 1), num(t, 2), num(t, 3));
            L->orientation = V3(num(t, 4), num(t, 5), num(t, 6));
            normalize_ip(L->orientation);
            L->lightColor = Color(num(t, 9), num(t, 10), num(t, 11));
            L->innerRad = num(t, 7) * DEG_TO_RAD_F;
            L->outerRad = num(t, 8) * DEG_TO_RAD_F;
            L->radDiff = L->outerRad - L->innerRad;
            L->oPhAxis = ortho_vec(L->orientation);
          } else {  // :435-444, myLight.java:244-247
            L->ltype = LT_DISK;
            L->origin = V3(num(t, 1), num(t, 2), num(t, 3));
            L->radius = num(t, 4);
            L->orientation = V3(num(t, 5), num(t, 6), num(t, 7));
            normalize_ip(L->orientation);
            L->lightColor = Color(num(t, 8), num(t, 9), num(t, 10));
            L->surfTangent = ortho_vec(L->orientation);
          }
          if (inTmpList) { err = "light inside accel list unsupported"; return false; }
          add_object(L);
        } else if (c == "caustic_photons" || c == "diffuse_photons") {  // setPhotonHandling :919-931
          s->usePhotonMap = true;
          s->isCausticPhtn = (c.find("caustic") != std::string::npos);
          s->photonTree.num_Cast = std::stoi(t.at(1));
          s->photonTree.maxNear = std::stoi(t.at(2));
          float md = std::stof(t.at(3));
          s->photonTree.baseMaxDist2 = (double)md * (double)md;
        } else if (c == "final_gather") {
        } else if (c == "diffuse") {
          txTop = txBtm = false;
          set_surface(Color(num(t, 1), num(t, 2), num(t, 3)), Color(num(t, 4), num(t, 5), num(t, 6)), Color(0, 0, 0), 0, 0);
        } else if (c == "reflective") {
          txTop = txBtm = false;
          set_surface(Color(num(t, 1), num(t, 2), num(t, 3)), Color(num(t, 4), num(t, 5), num(t, 6)), Color(0, 0, 0), 0, num(t, 7));
        } else if (c == "shiny" || c == "surface") {  // setSurfaceShiny :358-378
          Color d(num(t, 1), num(t, 2), num(t, 3)), a(num(t, 4), num(t, 5), num(t, 6)), sp(num(t, 7), num(t, 8), num(t, 9));
          double ph = num(t, 10), kr = num(t, 11), kt = 0, ri = 0;
          txTop = txBtm = false;
          set_surface(d, a, sp, ph, kr);
          if (t.size() > 12) {
            kt = num(t, 12);
            set_surface(d, a, sp, ph, kr); kTrans = kt;
            if (t.size() > 13) {
              ri = num(t, 13);
              rfrIdx = ri; permClr = Color(ri, ri, ri);
              if (t.size() > 16) permClr = Color(num(t, 14), num(t, 15), num(t, 16));
            }
          }
          if ((c == "shiny") && ((kt > 0) || (ri > 0))) simpleRefr = true;
        } else if (c == "perm") {
          rfrIdx = num(t, 1); permClr = Color(rfrIdx, rfrIdx, rfrIdx);
          if (t.size() > 4) permClr = Color(num(t, 2), num(t, 3), num(t, 4));
        } else if (c == "phong") { phong = num(t, 1);
        } else if (c == "krefl") { kRefl = num(t, 1); kReflClr = Color(kRefl, kRefl, kRefl);
        } else if (c == "ktrans") { kTrans = num(t, 1);
        } else if (c == "depth") {
        } else if (c == "begin_list") {
          inTmpList = true; tmpList.clear();
        } else if (c == "end_list" || c == "end_accel") {
          end_tmp_list(c == "end_accel");
        } else if (c == "named_object") {  // setObjectAsNamedObject (myScene.java:378-387)
          if (inTmpList || s->objList.empty()) { err = "named_object: no scene object to name"; return false; }
          GeomBase* o = s->objList.back();
          s->objList.pop_back();
          named[t.at(1)] = o;
        } else if (c == "instance") {  // myRTFileReader.java:250-256: any 3rd token selects the current shader
          if (!add_instance(t.at(1), t.size() > 2)) return false;
        } else if (c == "sierpinski") {  // myRTFileReader.java:234-241, buildSierpinski (myScene.java:371-377)
          std::string objName = t.at(1);
          float sc = .5f;
          int depth = 5;
          bool useShdr = false;  // useShdr != "No": true iff a 5th token was parsed
          try {
            depth = std::stoi(t.at(2));
            sc = std::stof(t.at(3));
            useShdr = t.size() > 4;
          } catch (...) {
          }
          if (inTmpList) { err = "sierpinski inside begin_list"; return false; }
          inTmpList = true; tmpList.clear();
          if (!sierp_sub(8, sc, objName, 0, depth, useShdr)) return false;
          end_tmp_list(true);
        } else if (c == "texture" || c == "image_texture") {
          std::string side = t.at(1), lo = side;
          for (auto& ch : lo) ch = (char)tolower(ch);
          if (lo == "top" || lo != "bottom") {
            texTopName = (lo == "top") ? t.at(2) : t.at(1);
            txTop = true;
          } else {
            txBtm = true;
          }
          txtrType = 1;
        } else if (c == "noise") {
          reset_dflt_txtr(); txtrType = 2; noiseScale = num(t, 1);
        } else if (c == "marble") {  // setTexture (myScene.java:712-777)
          reset_dflt_txtr();
          txtrType = 4;
          bool dflt = read_perlin(t);
          if (!useCustClrs) noiseColors = {Color(0.05, 0.05, 0.05), Color(0.95, 0.98, 0.92)};
          if (dflt) {
            numOctaves = 16; rndColors = true; useFwdTrans = false;
            noiseScale = 1.0; turbMult = 15.0; colorScale = 24.0; colorMult = .1;
            pdMult = V3(TWO_PI_F * 0.1, TWO_PI_F * 31.4, TWO_PI_F * 4.1);
          }
        } else if (c == "wood" || c == "wood2") {  // setTexture (myScene.java:717-742)
          reset_dflt_txtr();
          const bool w2 = c == "wood2";
          txtrType = w2 ? 6 : 3;
          bool dflt = read_perlin(t);
          if (!useCustClrs)
            noiseColors = w2 ? std::vector<Color>{Color(0.3, 0.20, 0.16), Color(0.94, 0.8, 0.4)}      // clr_dkwood2, clr_ltwood2
                             : std::vector<Color>{Color(0.2, 0.08, 0.08), Color(0.94, 0.47, 0.12)};  // clr_dkwood1, clr_ltwood1
          if (dflt) {
            numOctaves = w2 ? 8 : 4; rndColors = true; useFwdTrans = false;
            noiseScale = w2 ? 1.0 : 2.0; turbMult = .4; colorScale = 25.0; colorMult = w2 ? .3 : .2;
            pdMult = w2 ? V3(TWO_PI_F * 3.5, 7.9, 6.2) : V3(TWO_PI_F * 2.7, 3.6, 4.3);
          }
        } else if (c == "noise_color") {  // setTxtrColor (myScene.java:604-640); weights are unused by these textures
          if (!useCustClrs) { noiseColors.clear(); useCustClrs = true; }
          Color col;
          if (t.at(1) == "named") {
            if (!named_color(t.at(2), col)) { err = "unknown colour name: " + t.at(2); return false; }
          } else {
            col = Color(num(t, 1), num(t, 2), num(t, 3));
          }
          noiseColors.push_back(col);
        } else if (c == "stone") {  // setTexture (myScene.java:756-771)
          reset_dflt_txtr();
          txtrType = 5;
          bool dflt = read_worley(t);
          if (!useCustClrs)
            noiseColors = {Color(0.2, 0.2, 0.2), Color(0.7, 0.7, 0.7), Color(0.6, 0.18, 0.22), Color(0.8, 0.26, 0.33),
                           Color(0.6, 0.32, 0.16), Color(0.8, 0.45, 0.25), Color(0.3, 0.01, 0.07), Color(0.6, 0.02, 0.13),
                           Color(0.4, 0.1, 0.17), Color(0.6, 0.3, 0.13)};  // clr_mortar1/2, clr_brick1_1 .. clr_brick4_2
          if (dflt) {
            numOctaves = 8; numPtsDist = 2; distFunc = 1; roiFunc = 1; rndColors = true; useFwdTrans = false;
            noiseScale = 4.0; turbMult = 1.0; colorScale = 12.0; colorMult = .2; avgNumPerCell = 1.0; mortarThresh = 0.05;
            pdMult = V3(10.0, 10.0, 10.0);
          }
        } else if (c == "begin") {
          vertType = t.size() > 1 ? t[1] : "triangle";
          vc = 0;
          poly = s->make<Planar>();
          poly->ctm = cur_ctm();
          poly->vCount = (vertType == "quad") ? 4 : 3;
          poly->vx.assign(poly->vCount, 0); poly->vy.assign(poly->vCount, 0); poly->vz.assign(poly->vCount, 0);
          poly->vu.assign(poly->vCount, 0); poly->vv.assign(poly->vCount, 0);
          make_bbox(s, poly);
        } else if (c == "texture_coord") {
          poly->vu.at(vc) = num(t, 1); poly->vv.at(vc) = num(t, 2);
        } else if (c == "vertex") {
          poly->vx.at(vc) = num(t, 1); poly->vy.at(vc) = num(t, 2); poly->vz.at(vc) = num(t, 3);
          vc++;
        } else if (c == "end") {
          poly->finalize_poly();
          poly->shdr = cur_shader();
          poly->key = s->primCount++;
          add_object(poly);
          poly = nullptr;
          vertType = "triangle";
          vc = 0;
        } else if (c == "sphere" || c == "sphereIn" || c == "moving_sphere" || c == "ellipsoid") {  // readPrimData :447-521
          Sphere* sp = s->make<Sphere>();
          sp->ctm = cur_ctm();
          if (c == "ellipsoid") {
            sp->radX = num(t, 1); sp->radY = num(t, 2); sp->radZ = num(t, 3);
            sp->origin = V3(num(t, 4), num(t, 5), num(t, 6));
          } else {
            sp->radX = sp->radY = sp->radZ = num(t, 1);
            sp->origin = V3(num(t, 2), num(t, 3), num(t, 4));
          }
          if (c == "moving_sphere") {
            sp->moving = true;
            sp->origin0 = sp->origin;
            sp->origin1 = V3(num(t, 5), num(t, 6), num(t, 7));
          }
          sp->trans_origin = xpt(sp->ctm->g, sp->origin);
          sp->finalize_box();
          make_bbox(s, sp);
          if (c == "sphereIn") sp->inverted = true;
          sp->shdr = cur_shader();
          sp->key = s->primCount++;
          add_object(sp);
        } else if (c == "cyl" || c == "cylinder" || c == "hollow_cylinder") {
          double rad, hgt, xC, yC, zC, xO = 0, yO = 1, zO = 0;
          if (c == "cyl") {
            rad = num(t, 1); hgt = num(t, 2); xC = num(t, 3); yC = num(t, 4); zC = num(t, 5);
            if (t.size() > 8) { xO = num(t, 6); yO = num(t, 7); zO = num(t, 8); }
          } else {
            rad = num(t, 1); xC = num(t, 2); zC = num(t, 3); yC = num(t, 4); hgt = num(t, 5) - yC;
          }
          HollowCyl* cy;
          if (c == "hollow_cylinder") cy = s->make<HollowCyl>();
          else {
            Cyl* cc = s->make<Cyl>();
            cy = cc;
          }
          cy->ctm = cur_ctm();
          cy->radX = cy->radZ = rad; cy->myHeight = hgt;
          cy->origin = V3(xC, yC, zC);
          cy->yTop = cy->origin.y + hgt; cy->yBottom = cy->origin.y;
          if (c != "hollow_cylinder") {
            Cyl* cc = static_cast<Cyl*>(cy);
            cc->cap[0][0] = xO; cc->cap[0][1] = yO; cc->cap[0][2] = zO; cc->cap[0][3] = -cy->yTop;
            cc->cap[1][0] = xO; cc->cap[1][1] = -yO; cc->cap[1][2] = zO; cc->cap[1][3] = cy->yBottom;
          }
          cy->trans_origin = xpt(cy->ctm->g, cy->origin);
          cy->finalize_box();
          make_bbox(s, cy);
          cy->shdr = cur_shader();
          cy->key = s->primCount++;
          add_object(cy);
        } else if (c == "box") {
          double x0 = num(t, 1), y0 = num(t, 2), z0 = num(t, 3), x1 = num(t, 4), y1 = num(t, 5), z1 = num(t, 6);
          RndrdBox* b = s->make<RndrdBox>();
          b->ctm = cur_ctm();
          V3 mn(jmin(x0, x1), jmin(y0, y1), jmin(z0, z1)), mx(jmax(x0, x1), jmax(y0, y1), jmax(z0, z1));
          // p.min/p.max over 2 values skip NaN; jmin/jmax equal for finite input
          b->origin = V3((mn.x + mx.x) * .5, (mn.y + mx.y) * .5, (mn.z + mx.z) * .5);
          b->trans_origin = xpt(b->ctm->g, b->origin);
          b->minVals = mn; b->maxVals = mx;
          make_bbox(s, b);
          b->shdr = cur_shader();
          b->key = s->primCount++;
          add_object(b);
        } else if (c == "plane") {  // myPlane.setPlaneVals (myPlanarObject.java:236-270)
          Planar* pl = s->make<Planar>();
          pl->ctm = cur_ctm();
          pl->isPlane = true;
          pl->vCount = 4;
          pl->vx.assign(4, 0); pl->vy.assign(4, 0); pl->vz.assign(4, 0); pl->vu.assign(4, 0); pl->vv.assign(4, 0);
          make_bbox(s, pl);
          double a = num(t, 1), b = num(t, 2), cc = num(t, 3), d = num(t, 4);
          V3 N(a, b, cc);
          double m = mag(N);
          normalize_ip(N);
          double pA = N.x, pB = N.y, pC = N.z, pD = d / m;
          V3 rot(pB, pC, pA);
          if ((pA == pB) && (pA == pC)) rot = V3(rot.x + 1, rot.y, rot.z);
          normalize_ip(rot);
          int idx = 7;
          double sum = pA + pB + pC;
          if (sum == 0) { sum = pA + pB; idx = 6; if (sum == 0) { sum = pA + pC; idx = 5; if (sum == 0) { sum = pB + pC; idx = 3; } } }
          V3 pp(((idx & 4) == 4 ? -pD / sum : 0), ((idx & 2) == 2 ? -pD / sum : 0), ((idx & 1) == 1 ? -pD / sum : 0));
          V3 inU = cross(N, rot), inV = cross(N, inU);
          pl->vx[0] = pp.x; pl->vy[0] = pp.y; pl->vz[0] = pp.z;
          V3 np(pp.x + inU.x, pp.y + inU.y, pp.z + inU.z);
          pl->vx[1] = np.x; pl->vy[1] = np.y; pl->vz[1] = np.z;
          np = V3(np.x + inV.x, np.y + inV.y, np.z + inV.z);
          pl->vx[2] = np.x; pl->vy[2] = np.y; pl->vz[2] = np.z;
          np = V3(pp.x + inV.x, pp.y + inV.y, pp.z + inV.z);
          pl->vx[3] = np.x; pl->vy[3] = np.y; pl->vz[3] = np.z;
          pl->origin = pp;
          // state A: N/D from setPlaneVals; state B: invertNormal from the 4 vertices
          PlanarState& A = pl->st[0];
          A.vx = pl->vx; A.vy = pl->vy; A.vz = pl->vz; A.vu = pl->vu; A.vv = pl->vv;
          Planar::set_points_and_normal(A, 4);
          A.N = N; A.D = pD;
          pl->build_reversed();
          pl->shdr = cur_shader();
          pl->key = s->primCount++;
          add_object(pl);
        } else if (c == "push") {
          push();
        } else if (c == "pop") {
          pop();
        } else if (c == "translate") {
          translate(num(t, 1), num(t, 2), num(t, 3));
        } else if (c == "scale") {
          scale(num(t, 1), num(t, 2), num(t, 3));
        } else if (c == "rotate") {
          rotate(num(t, 1), num(t, 2), num(t, 3), num(t, 4));
        } else if (c == "reset_timer" || c == "print_timer" || c == "refine") {
          // timers and the progressive `refine` preview are ignored (documented override)
        } else {
          // myRTFileReader.java:343-345: the default case prints the line and reading goes on
          ++ignored;
        }
      } catch (const std::exception& e) {
        err = "parse error in " + fname + " at command '" + c + "': " + e.what();
        return false;
      }
    }
    return true;
  }
};

}  // namespace orc

// ---------------------------------------------------------------------------
// C API (consumed by tests/ via ctypes)
using namespace orc;
static std::map<std::string, Texture> g_textures;
static std::string g_err;

extern "C" {

const char* oracle_last_error() { return g_err.c_str(); }

int oracle_register_texture(const char* name, int w, int h, const uint8_t* rgb) {
  Texture t;
  t.w = w; t.h = h;
  t.px.resize((size_t)w * h);
  for (size_t i = 0; i < t.px.size(); ++i)
    t.px[i] = 0xFF000000u | ((uint32_t)rgb[3 * i] << 16) | ((uint32_t)rgb[3 * i + 1] << 8) | (uint32_t)rgb[3 * i + 2];
  g_textures[name] = std::move(t);
  return 0;
}

void* oracle_load(const char* dir, const char* file) {
  Scene* s = new Scene();
  s->textures = &g_textures;
  Loader L;
  L.s = s;
  L.dir = dir;
  if (!L.read_file(file, true) || !L.err.empty()) {
    g_err = L.err;
    delete s;
    return nullptr;
  }
  return s;
}

void oracle_free(void* p) { delete (Scene*)p; }

// info[0..]: numObjs, numLights, bvhInternal, bvhLeaves, bvhDepth, bvhPrims, primCount, numRaysPerPixel
int oracle_info(void* p, int64_t* info, int n) {
  Scene* s = (Scene*)p;
  int64_t v[8] = {(int64_t)s->objList.size(), (int64_t)s->lightList.size(), s->bvhInternal, s->bvhLeaves, s->bvhDepth,
                  s->bvhPrims, (int64_t)s->primCount, s->numRaysPerPixel};
  for (int i = 0; i < n && i < 8; ++i) info[i] = v[i];
  return 0;
}

int oracle_build_photons(void* p, uint64_t seed) {
  Scene* s = (Scene*)p;
  if (s->usePhotonMap) send_photons(s, seed);
  return (int)s->photonTree.photons.size();
}

// photon_list in insertion order (test access): pos/pwr = double[n*3]; returns the count
int oracle_photons(void* p, double* pos, double* pwr, int n) {
  Scene* s = (Scene*)p;
  const std::vector<Photon>& ph = s->photonTree.photons;
  for (int i = 0; i < n && i < (int)ph.size(); ++i)
    for (int c = 0; c < 3; ++c) { pos[3 * i + c] = ph[i].pos[c]; pwr[3 * i + c] = ph[i].pwr[c]; }
  return (int)ph.size();
}

// Render rows [row0,row1) with stride rowStep of a W x H image (myFOVScene.draw,
// myScene.java:1481-1531 + DOF :1386-1443). spp<=0 keeps the scene's
// rays_per_pixel. rgb: float[nrows*W*3], argb: int32[nrows*W]; stats: uint64[16].
int oracle_render(void* p, int W, int H, int spp, uint64_t seed, int row0, int row1, int rowStep, float* rgb,
                  int32_t* argb, uint64_t* stats, int nthreads) {
  Scene* s = (Scene*)p;
  s->W = W; s->H = H;
  if (spp > 0) s->numRaysPerPixel = spp;
  if (s->usePhotonMap && !s->photonsBuilt) send_photons(s, seed);
  double fovRad = M_PI * s->fov / 180.0;
  if (std::fabs(s->fov - 180) < .001) fovRad -= .0001;
  s->viewZ = -1 * (std::max(H, W) / 2.0) / std::tan(fovRad / 2);
  if (s->hasDOF && !s->focalPlane) {  // focal plane z = -focal (myScene.java:805-810)
    Planar* fp = s->make<Planar>();
    fp->ctm = std::make_shared<CTM>(build_ctm(M4()));
    fp->isPlane = true; fp->vCount = 4;
    PlanarState& A = fp->st[0];
    A.N = V3(0, 0, 1); A.D = s->lensFocal;
    fp->st[1] = A; fp->st[1].N = V3(0, 0, -1); fp->st[1].D = -s->lensFocal;
    s->focalPlane = fp;
  }
  double rayYOffset = H / 2.0, rayXOffset = W / 2.0;
  int nrows = 0;
  for (int r = row0; r < row1; r += rowStep) nrows++;
  std::vector<std::vector<uint64_t>> tst(nthreads > 0 ? nthreads : 1, std::vector<uint64_t>(ST_N, 0));
  int n = s->numRaysPerPixel;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int ri = 0; ri < nrows; ++ri) {
#ifdef _OPENMP
    uint64_t* st = tst[omp_get_thread_num()].data();
#else
    uint64_t* st = tst[0].data();
#endif
    int row = row0 + ri * rowStep;
    double rayY = (-1 * (row - rayYOffset));
    for (int col = 0; col < W; ++col) {
      double rayX = col - rayXOffset;
      uint64_t pix = (uint64_t)row * (uint64_t)W + (uint64_t)col;
      Color c;
      if (s->camType == 1) {  // myFishEyeScene.draw / shootMultiRays (myScene.java:1562-1653)
        const double maxDim = std::max(H, W);
        const double yStart = ((maxDim - H) / 2.0) - rayYOffset, xStart = ((maxDim - W) / 2.0) - rayXOffset;
        const double fishMult = 2.0 / maxDim;  // setImageSize :780-792
        const double aperatureHlf = (M_PI * s->fishEye / 180.0) / 2.0;
        auto fish_ray = [&](double xVal, double yVal, double rSq, uint32_t k) -> Color {
          double r = std::sqrt(rSq), theta = r * aperatureHlf, phi = std::atan2(-yVal, xVal), sTh = jf::sin(theta);
          Ray ray(V3(0, 0, 0), V3(sTh * jf::cos(phi), sTh * jf::sin(phi), -jf::cos(theta)), 0);
          ray.key.seed = seed; ray.key.pixel = pix; ray.key.sample = k; ray.key.node = 1;
          st[ST_CAM]++;
          return reflect_ray(s, ray, st);
        };
        if (n == 1) {
          double yVal = (row + yStart) * fishMult, ySq = yVal * yVal, xVal = (col + xStart) * fishMult;
          double rTmp = xVal * xVal + ySq;
          c = (rTmp > 1) ? Color(0, 0, 0) : fish_ray(xVal, yVal, rTmp, 0);  // blkColor outside the circle
        } else {
          double yB = row + yStart, xB = col + xStart, rs = 0, gs = 0, bs = 0;
          for (int k = 0; k < n; ++k) {
            double yVal = (yB + rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_Y, 0), -.5, .5)) * fishMult;
            double xVal = (xB + rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_X, 0), -.5, .5)) * fishMult;
            double rSq = yVal * yVal + xVal * xVal;
            if (rSq <= 1) {
              Color cc = fish_ray(xVal, yVal, rSq, (uint32_t)k);
              rs += cc.r; gs += cc.g; bs += cc.b;
            }
          }
          c = Color(rs / n, gs / n, bs / n);
        }
      } else if (s->camType == 2) {  // myOrthoScene.draw / shootMultiRays (myScene.java:1690-1753)
        const double div = std::min(W, H);  // the reference divides by the applet's (= image) size
        const double orthPerRow = s->orthoH / div, orthPerCol = s->orthoW / div;
        auto ortho_ray = [&](double rx, double ry, uint32_t k) -> Color {
          Ray ray(V3(rx, ry, 0), V3(0, 0, -1), 0);
          ray.key.seed = seed; ray.key.pixel = pix; ray.key.sample = k; ray.key.node = 1;
          st[ST_CAM]++;
          return reflect_ray(s, ray, st);
        };
        if (n == 1) {
          c = ortho_ray(orthPerCol * (col - rayXOffset), orthPerRow * (-1 * (row - rayYOffset)), 0);
        } else {
          double yB = orthPerRow * ((-1 * (row - rayYOffset)) - .5), xB = orthPerCol * (col - rayXOffset - .5);
          double rs = 0, gs = 0, bs = 0;
          for (int k = 0; k < n; ++k) {
            double ry = yB + (orthPerRow * rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_Y, 0), -.5, .5));
            double rx = xB + (orthPerCol * rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_X, 0), -.5, .5));
            Color cc = ortho_ray(rx, ry, (uint32_t)k);
            rs += cc.r; gs += cc.g; bs += cc.b;
          }
          c = Color(rs / n, gs / n, bs / n);
        }
      } else if (s->hasDOF) {  // shootMultiDpthOfFldRays :1386-1406
        V3 lc(rayX, rayY, s->viewZ);
        normalize_ip(lc);
        Ray ray(V3(0, 0, 0), lc, 0);
        Ray tr = transformed(ray, s->focalPlane->ctm->inv, 0);
        Hit fh = s->focalPlane->intersect(ray, tr, s->focalPlane->ctm.get(), nullptr);
        V3 fpt = fh.hitLoc;
        double rs = 0, gs = 0, bs = 0;
        for (int k = 0; k < n; ++k) {
          V3 t = rot_around_axis(V3(0, 1, 0), V3(0, 0, -1), rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_DOF_ANG, 0), 0, TWO_PI_F));
          normalize_ip(t);
          double m = rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_DOF_RAD, 0), 0, s->lensRadius);
          t = V3(t.x * m, t.y * m, t.z * m);
          V3 o(t.x + lc.x, t.y + lc.y, t.z + lc.z);
          Ray r(o, vsub(fpt, o), 0);
          r.key.seed = seed; r.key.pixel = pix; r.key.sample = (uint32_t)k; r.key.node = 1;
          st[ST_CAM]++;
          Color cc = reflect_ray(s, r, st);
          rs += cc.r; gs += cc.g; bs += cc.b;
        }
        c = Color(rs / n, gs / n, bs / n);
      } else if (n == 1) {
        Ray r(V3(0, 0, 0), V3(rayX, rayY, s->viewZ), 0);
        r.key.seed = seed; r.key.pixel = pix; r.key.sample = 0; r.key.node = 1;
        st[ST_CAM]++;
        c = reflect_ray(s, r, st);
      } else {  // shootMultiRays :1447-1462 (y jitter drawn before x)
        double rs = 0, gs = 0, bs = 0;
        for (int k = 0; k < n; ++k) {
          double ry = rayY + rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_Y, 0), -.5, .5);
          double rx = rayX + rng_range(rng_bits(seed, pix, (uint32_t)k, 0, SITE_AA_X, 0), -.5, .5);
          Ray r(V3(0, 0, 0), V3(rx, ry, s->viewZ), 0);
          r.key.seed = seed; r.key.pixel = pix; r.key.sample = (uint32_t)k; r.key.node = 1;
          st[ST_CAM]++;
          Color cc = reflect_ray(s, r, st);
          rs += cc.r; gs += cc.g; bs += cc.b;
        }
        c = Color(rs / n, gs / n, bs / n);
      }
      size_t o = (size_t)ri * W + col;
      if (rgb) { rgb[3 * o] = (float)c.r; rgb[3 * o + 1] = (float)c.g; rgb[3 * o + 2] = (float)c.b; }
      if (argb) argb[o] = color_argb(c);
    }
  }
  if (stats)
    for (auto& v : tst)
      for (int i = 0; i < ST_N; ++i) stats[i] += v[i];
  return 0;
}

// Install a photon_list (insertion order; e.g. the product's rt_scene_photons output) and build
// the oracle's own kd-tree over it (myKD_Tree.build_tree, myLight.java:325-381), so both sides
// gather over the identical list (tests/test_gpu_parity.py C5 at k = 200).
int oracle_set_photons(void* p, const double* pos, const double* pwr, int64_t n) {
  Scene* s = (Scene*)p;
  KDTree& T = s->photonTree;
  T.photons.assign((size_t)n, Photon{});
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) { T.photons[i].pos[c] = pos[3 * i + c]; T.photons[i].pwr[c] = pwr[3 * i + c]; }
  T.build_all();
  s->photonsBuilt = true;
  return 0;
}

// The photon neighbourhood find_near returns for a point (myKD_Tree.find_near, myLight.java:389-445):
// up to cap photon indices (photon_list order) in poll order, farthest first, and their d2; returns
// the neighbourhood's size. Tests check the JDK 8 PriorityQueue tie rules on it.
int oracle_knn(void* p, double x, double y, double z, int32_t* idx, double* d2, int cap) {
  Scene* s = (Scene*)p;
  std::vector<KDTree::QE> out;
  s->photonTree.find_near(V3(x, y, z), out, nullptr);
  for (int i = 0; i < (int)out.size() && i < cap; ++i) { idx[i] = out[i].p; d2[i] = out[i].d2; }
  return (int)out.size();
}

// fdlibm sin / cos / asin / acos (jfdlibm.h, shared with the device) of x[0..n) -> out[4*i..4*i+3]
int oracle_math_eval(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    out[4 * i + 0] = jf::sin(x[i]); out[4 * i + 1] = jf::cos(x[i]);
    out[4 * i + 2] = jf::asin(x[i]); out[4 * i + 3] = jf::acos(x[i]);
  }
  return 0;
}

// Camera-ray hit mask of a W x H FOV render at 1 spp (myFOVScene.draw, myScene.java:1498-1508):
// mask[row*W+col] = 1 where the un-jittered camera ray hits an object, 0 where it falls through
// to the background / skydome (reflectRay, :907-914). Used to derive the sky-pixel fixture pinned
// to the reference's own t11_sierp.png (tests/golden/make_sky_pin.py).
int oracle_camera_hits(void* p, int W, int H, uint8_t* mask, int nthreads) {
  Scene* s = (Scene*)p;
  if (s->camType != 0 || s->hasDOF) { g_err = "oracle_camera_hits: FOV camera without lens only"; return -1; }
  double fovRad = M_PI * s->fov / 180.0;
  if (std::fabs(s->fov - 180) < .001) fovRad -= .0001;
  const double viewZ = -1 * (std::max(H, W) / 2.0) / std::tan(fovRad / 2);
  const double rayYOffset = H / 2.0, rayXOffset = W / 2.0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int row = 0; row < H; ++row) {
    uint64_t st[ST_N] = {0};
    for (int col = 0; col < W; ++col) {
      Ray r(V3(0, 0, 0), V3(col - rayXOffset, (-1 * (row - rayYOffset)), viewZ), 0);
      r.key.pixel = (uint64_t)row * (uint64_t)W + (uint64_t)col; r.key.sample = 0; r.key.node = 1;
      mask[(size_t)row * W + col] = closest_hit(s, r, st).isHit ? 1 : 0;
    }
  }
  return 0;
}

}  // extern "C"
