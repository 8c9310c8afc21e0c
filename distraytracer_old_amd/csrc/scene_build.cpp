// rt_scene_desc -> flattened HostScene (rt_types.h), the layout the HIP
// kernels read from HBM. Precomputes, with the reference's arithmetic:
//  * CTM arrays [g, inv, trans, adj] (DistRayTracer.java:399-405),
//  * planar equations for BOTH vertex orders (myPlanarObject.java:44-100),
//  * object boxes (postProcBBox, myGeomBase.java:42-45, per-type getMin/MaxVec),
//  * trans_origin centroids (myGeomBase.java:39, myPlanarObject.java:67-68),
//  * BVHs with the reference topology: object-median split on the axis of max
//    centroid span, stable per-axis orders, leaf <= 5, root built with
//    endIDX = N-1 (Q1: last element of the root's split-axis order dropped)
//    (myScene.java:312-318, myGeomBase.java:338-386, DistRayTracer.java:409-418).
#include <algorithm>
#include <cmath>
#include <map>
#include <string>

#include "host_math.h"
#include "rt_internal.h"

namespace rt {
using namespace hm;

namespace {

struct Box {
  double mn[3] = {100000, 100000, 100000};  // myGeomBase ctor defaults (:35-36)
  double mx[3] = {-100000, -100000, -100000};
};
// myBBox.calcMinMaxCtrVals (myGeomBase.java:102-104)
static void calc_min_max(Box& b, const double* mn, const double* mx) {
  for (int i = 0; i < 3; ++i) { b.mn[i] = jmin(mn[i], b.mn[i]); b.mx[i] = jmax(mx[i], b.mx[i]); }
}
// expandBoxPt (DistRayTracer.java:353-361)
static void expand_pt(Box& b, D3 p) {
  double v[3] = {p.x, p.y, p.z};
  for (int i = 0; i < 3; ++i) {
    b.mn[i] = (b.mn[i] < v[i]) ? b.mn[i] : v[i];
    b.mx[i] = (b.mx[i] > v[i]) ? b.mx[i] : v[i];
  }
}
static void expand_box(Box& t, const Box& s, const Mat* fwd) {  // expandBoxByBox :364-371
  D3 a = d3(s.mn[0], s.mn[1], s.mn[2]), b = d3(s.mx[0], s.mx[1], s.mx[2]);
  if (fwd) { a = xform(*fwd, a, 1); b = xform(*fwd, b, 1); }
  expand_pt(t, a);
  expand_pt(t, b);
}

struct PlanarEq {
  D3 N;
  double D;
};
// setPointsAndNormal + setEQ for a vertex order (myPlanarObject.java:44-69,90)
static PlanarEq planar_eq(const double (*v)[3], int n) {
  std::vector<D3> P2P(n);
  for (int i = 0; i < n; i++) {
    int idx = (i != 0 ? i - 1 : n - 1);
    P2P[idx] = d3(v[i][0] - v[idx][0], v[i][1] - v[idx][1], v[i][2] - v[idx][2]);
  }
  PlanarEq e;
  e.N = normalized(cross(P2P[1], P2P[0]));
  e.D = -((e.N.x * v[0][0]) + (e.N.y * v[0][1]) + (e.N.z * v[0][2]));
  return e;
}

struct Builder {
  const rt_scene_desc* d;
  HostScene& hs;
  std::map<std::string, int> xfIndex;
  // object ids: desc prim i -> i, desc instance j -> num_prims + j
  std::vector<int32_t> ref;      // object -> encoded ref (>=0 tri, <0 ~prim; instances are PT_INST prims)
  std::vector<D3> transOrigin;   // object -> CTM * origin
  std::vector<Box> objBox;       // object -> object-space bbox (_bbox)
  std::vector<char> boxReady;    // instance boxes are formed when an accel first needs them
  std::vector<char> accHasInst, instUsed;
  std::string err;

  Builder(const rt_scene_desc* dd, HostScene& h) : d(dd), hs(h) {}

  int xf_id(const Mat& g) {
    std::string k((const char*)g.m, sizeof(g.m));
    auto it = xfIndex.find(k);
    if (it != xfIndex.end()) return it->second;
    XformD x;
    Mat inv = inverse(g), adj = transpose(inv);
    std::memcpy(x.g, g.m, sizeof(x.g));
    std::memcpy(x.inv, inv.m, sizeof(x.inv));
    std::memcpy(x.adj, adj.m, sizeof(x.adj));
    hs.xf.push_back(x);
    int id = (int)hs.xf.size() - 1;
    xfIndex[k] = id;
    return id;
  }
  static Mat ctm_of(const double* m) {
    Mat r;
    std::memcpy(r.m, m, sizeof(r.m));
    return r;
  }

  bool build_prim(int i) {
    const rt_prim_desc& p = d->prims[i];
    Mat g = ctm_of(p.ctm);
    int xf = xf_id(g);
    Box bb;
    D3 origin = d3(0, 0, 0);
    if (p.type == RT_PRIM_TRIANGLE || p.type == RT_PRIM_QUAD) {
      int n = p.type == RT_PRIM_TRIANGLE ? 3 : 4;
      double rv[4][3];
      for (int k = 0; k < n; ++k) for (int c = 0; c < 3; ++c) rv[n - 1 - k][c] = p.v[k][c];
      PlanarEq A = planar_eq(p.v, n), B = planar_eq(rv, n);
      double sx = 0, sy = 0, sz = 0;
      for (int k = 0; k < n; ++k) { sx += p.v[k][0]; sy += p.v[k][1]; sz += p.v[k][2]; }
      origin = d3(sx / n, sy / n, sz / n);
      double mn[3], mx[3];  // p.min / p.max over vertices (NaN-skipping, DistRayTracer.java:424-425)
      for (int c = 0; c < 3; ++c) {
        mn[c] = DMAX; mx[c] = -DMAX;
        for (int k = 0; k < n; ++k) { if (p.v[k][c] < mn[c]) mn[c] = p.v[k][c]; if (p.v[k][c] > mx[c]) mx[c] = p.v[k][c]; }
      }
      calc_min_max(bb, mn, mx);
      if (n == 3) {
        if (!(B.N.x == -A.N.x && B.N.y == -A.N.y && B.N.z == -A.N.z) &&
            !(A.N.x != A.N.x || A.N.y != A.N.y || A.N.z != A.N.z)) {
          err = "internal: triangle reversed normal is not exactly -N";
          return false;
        }
        TriD t;
        std::memset(&t, 0, sizeof(t));
        for (int k = 0; k < 3; ++k) for (int c = 0; c < 3; ++c) t.v[k][c] = p.v[k][c];
        t.n[0] = A.N.x; t.n[1] = A.N.y; t.n[2] = A.N.z;
        t.dA = A.D; t.dB = B.D;
        t.xf = xf; t.xfc = -1; t.mat = p.material; t.key = (uint32_t)i;
        hs.tri.push_back(t);
        for (int k = 0; k < 3; ++k) { hs.triUV.push_back(p.uv[k][0]); hs.triUV.push_back(p.uv[k][1]); }
        ref[i] = (int32_t)hs.tri.size() - 1;
      } else {
        PrimD q;
        std::memset(&q, 0, sizeof(q));
        q.type = PT_QUAD;
        for (int k = 0; k < 4; ++k) for (int c = 0; c < 3; ++c) q.a[3 * k + c] = p.v[k][c];
        q.a[12] = A.N.x; q.a[13] = A.N.y; q.a[14] = A.N.z;
        q.a[15] = B.N.x; q.a[16] = B.N.y; q.a[17] = B.N.z;
        q.a[18] = A.D; q.a[19] = B.D;
        for (int k = 0; k < 4; ++k) { q.a[20 + 2 * k] = p.uv[k][0]; q.a[21 + 2 * k] = p.uv[k][1]; }
        push_prim(q, i, xf, p);
      }
    } else if (p.type == RT_PRIM_PLANE) {  // myPlane.setPlaneVals (myPlanarObject.java:236-270)
      D3 N = d3(p.p[0], p.p[1], p.p[2]);
      double m = std::sqrt(((N.x * N.x) + (N.y * N.y)) + (N.z * N.z));
      N = normalized(N);
      double pA = N.x, pB = N.y, pC = N.z, pD = p.p[3] / m;
      D3 rot = d3(pB, pC, pA);
      if ((pA == pB) && (pA == pC)) rot.x = rot.x + 1;
      rot = normalized(rot);
      int idx = 7;
      double sum = pA + pB + pC;
      if (sum == 0) { sum = pA + pB; idx = 6; if (sum == 0) { sum = pA + pC; idx = 5; if (sum == 0) { sum = pB + pC; idx = 3; } } }
      D3 pp = d3(((idx & 4) == 4 ? -pD / sum : 0), ((idx & 2) == 2 ? -pD / sum : 0), ((idx & 1) == 1 ? -pD / sum : 0));
      D3 inU = cross(N, rot), inV = cross(N, inU);
      double v[4][3], rv[4][3];
      D3 np = d3(pp.x + inU.x, pp.y + inU.y, pp.z + inU.z);
      D3 np2 = d3(np.x + inV.x, np.y + inV.y, np.z + inV.z);
      D3 np3 = d3(pp.x + inV.x, pp.y + inV.y, pp.z + inV.z);
      D3 vs[4] = {pp, np, np2, np3};
      for (int k = 0; k < 4; ++k) { v[k][0] = vs[k].x; v[k][1] = vs[k].y; v[k][2] = vs[k].z; }
      for (int k = 0; k < 4; ++k) for (int c = 0; c < 3; ++c) rv[3 - k][c] = v[k][c];
      PlanarEq B = planar_eq(rv, 4);
      PrimD q;
      std::memset(&q, 0, sizeof(q));
      q.type = PT_PLANE;
      for (int k = 0; k < 4; ++k) for (int c = 0; c < 3; ++c) q.a[3 * k + c] = v[k][c];
      q.a[12] = N.x; q.a[13] = N.y; q.a[14] = N.z;
      q.a[15] = B.N.x; q.a[16] = B.N.y; q.a[17] = B.N.z;
      q.a[18] = pD; q.a[19] = B.D;
      origin = d3(0, 0, 0);  // trans_origin is computed in the myGeomBase ctor, before setPlaneVals
      push_prim(q, i, xf, p);
    } else if (p.type == RT_PRIM_SPHERE || p.type == RT_PRIM_MOVING_SPHERE) {
      PrimD q;
      std::memset(&q, 0, sizeof(q));
      q.type = p.type == RT_PRIM_SPHERE ? PT_SPHERE : PT_MSPHERE;
      for (int k = 0; k < 9; ++k) q.a[k] = p.p[k];
      q.flags = (p.flags & RT_PRIM_INVERTED) ? 1 : 0;
      origin = d3(p.p[0], p.p[1], p.p[2]);
      double tv = p.p[3] + p.p[4] + p.p[5];  // L1 half-extent (myImpObject.java:127-139, Q16)
      double mn[3] = {origin.x + -tv, origin.y + -tv, origin.z + -tv}, mx[3] = {origin.x + tv, origin.y + tv, origin.z + tv};
      calc_min_max(bb, mn, mx);
      push_prim(q, i, xf, p);
    } else if (p.type == RT_PRIM_CYLINDER || p.type == RT_PRIM_HOLLOW_CYLINDER) {
      PrimD q;
      std::memset(&q, 0, sizeof(q));
      q.type = p.type == RT_PRIM_CYLINDER ? PT_CYL : PT_HCYL;
      double r = p.p[0], h = p.p[1];
      origin = d3(p.p[2], p.p[3], p.p[4]);
      q.a[0] = origin.x; q.a[1] = origin.y; q.a[2] = origin.z;
      q.a[3] = r; q.a[4] = r; q.a[5] = h;
      q.a[6] = origin.y + h;  // yTop
      q.a[7] = origin.y;      // yBottom
      double ox = p.p[5], oy = p.p[6], oz = p.p[7];
      q.a[8] = ox; q.a[9] = oy; q.a[10] = oz; q.a[11] = -q.a[6];    // top cap
      q.a[12] = ox; q.a[13] = -oy; q.a[14] = oz; q.a[15] = q.a[7];  // bottom cap
      double tv = r + r;
      double mn[3] = {origin.x + -tv, origin.y + 0, origin.z + -tv}, mx[3] = {origin.x + tv, origin.y + h, origin.z + tv};
      calc_min_max(bb, mn, mx);
      push_prim(q, i, xf, p);
    } else if (p.type == RT_PRIM_BOX) {  // readPrimData "box" (myScene.java:450-462)
      PrimD q;
      std::memset(&q, 0, sizeof(q));
      q.type = PT_BOX;
      double mn[3], mx[3];
      for (int c = 0; c < 3; ++c) {
        double a = p.p[c], b = p.p[3 + c];
        mn[c] = (a != a) ? b : ((b != b) ? a : (b < a ? b : a));
        mx[c] = (a != a) ? b : ((b != b) ? a : (b > a ? b : a));
        q.a[c] = mn[c]; q.a[3 + c] = mx[c];
      }
      origin = d3((mn[0] + mx[0]) * .5, (mn[1] + mx[1]) * .5, (mn[2] + mx[2]) * .5);
      calc_min_max(bb, mn, mx);
      push_prim(q, i, xf, p);
    } else {
      err = "unknown primitive type";
      return false;
    }
    transOrigin[i] = xform(g, origin, 1);
    objBox[i] = bb;
    return true;
  }
  void push_prim(PrimD& q, int i, int xf, const rt_prim_desc& p) {
    q.xf = xf; q.xfc = -1; q.mat = p.material; q.key = (uint32_t)i;
    hs.prim.push_back(q);
    ref[i] = ~(int32_t)(hs.prim.size() - 1);
  }
  const double* obj_ctm(int id) const {
    return id < d->num_prims ? d->prims[id].ctm : d->instances[id - d->num_prims].ctm;
  }
  // desc member / top entry -> object id (-1: out of range)
  int obj_id(int32_t m) const {
    if (m >= 0 && (m & RT_REF_INSTANCE)) {
      int j = m & ~RT_REF_INSTANCE;
      return j < d->num_instances ? d->num_prims + j : -1;
    }
    return (m >= 0 && m < d->num_prims) ? m : -1;
  }
  // myInstance (mySceneObject.java:98-110): a PT_INST prim naming the object
  bool build_instance(int j) {
    const rt_instance_desc& in = d->instances[j];
    PrimD q;
    std::memset(&q, 0, sizeof(q));
    q.type = PT_INST;
    q.xf = xf_id(ctm_of(in.ctm));
    q.xfc = -1;
    if (in.material < -1 || in.material >= d->num_materials) { err = "instance: bad material index"; return false; }
    q.mat = in.material;
    if (in.base >= 0) {
      if (in.base >= d->num_prims) { err = "instance: base prim out of range"; return false; }
      int ty = d->prims[in.base].type;
      if (ty != RT_PRIM_TRIANGLE && ty != RT_PRIM_QUAD && ty != RT_PRIM_SPHERE && ty != RT_PRIM_CYLINDER &&
          ty != RT_PRIM_HOLLOW_CYLINDER) {
        err = "instance: unsupported named primitive (plane / box / moving sphere)";
        return false;
      }
      q.pad[0] = ref[in.base];
      q.key = (uint32_t)in.base;
    } else {
      int ai = ~in.base;
      if (ai >= d->num_accels) { err = "instance: base accel out of range"; return false; }
      q.flags = PF_INST_ACCEL;
      q.pad[0] = ai;
    }
    hs.prim.push_back(q);
    const int id = d->num_prims + j;
    ref[id] = ~(int32_t)(hs.prim.size() - 1);
    transOrigin[id] = d3(in.origin[0], in.origin[1], in.origin[2]);
    return true;
  }
  // the instance's _bbox: named object's getMin/MaxVec through its own CTM (mySceneObject.java:104-113)
  bool instance_box(int id, int curAccel) {
    if (boxReady[id]) return true;
    const rt_instance_desc& in = d->instances[id - d->num_prims];
    Box base;
    if (in.base >= 0) {
      base = objBox[in.base];
    } else {
      int ai = ~in.base;
      if (ai >= curAccel) { err = "instance of an accel defined later"; return false; }
      if (accHasInst[ai]) { err = "instance of an accel holding instances is unsupported"; return false; }
      const AccelD& a = hs.accel[ai];
      for (int c = 0; c < 3; ++c) { base.mn[c] = a.bmin[c]; base.mx[c] = a.bmax[c]; }
    }
    Mat bg = ctm_of(in.base >= 0 ? d->prims[in.base].ctm : d->accels[~in.base].ctm);
    D3 mn = xform(bg, d3(base.mn[0], base.mn[1], base.mn[2]), 1), mx = xform(bg, d3(base.mx[0], base.mx[1], base.mx[2]), 1);
    double a[3] = {mn.x, mn.y, mn.z}, b[3] = {mx.x, mx.y, mx.z};
    Box bb;
    calc_min_max(bb, a, b);
    objBox[id] = bb;
    boxReady[id] = 1;
    return true;
  }
  void set_xfc(int i, int xfc) {
    int32_t r = ref[i];
    if (r >= 0) hs.tri[r].xfc = xfc;
    else hs.prim[~r].xfc = xfc;
  }

  // ---- BVH (myBVH.addObjList) -------------------------------------------
  typedef std::vector<int> L;
  void sorted(const L& in, int axis, L& out) {
    out = in;
    std::stable_sort(out.begin(), out.end(), [&](int a, int b) {
      double va = axis == 0 ? transOrigin[a].x : (axis == 1 ? transOrigin[a].y : transOrigin[a].z);
      double vb = axis == 0 ? transOrigin[b].x : (axis == 1 ? transOrigin[b].y : transOrigin[b].z);
      return jcompare(va, vb) < 0;
    });
  }
  double comp(int p, int ax) { return ax == 0 ? transOrigin[p].x : (ax == 1 ? transOrigin[p].y : transOrigin[p].z); }
  // returns child ref; box = node's _bbox
  int32_t bvh(L lists[3], int st, int en, int depth, const Mat& accInv, int accXf, Box& box) {
    int sz = en - st;
    if (sz <= 5) {
      Box lb;  // leafVals._bbox
      LeafD lf;
      lf.start = (int)hs.member.size();
      lf.count = (int)lists[0].size();
      for (int p : lists[0]) {
        Mat tmp = mul(accInv, ctm_of(obj_ctm(p)));
        expand_box(lb, objBox[p], &tmp);
        hs.member.push_back(ref[p]);
      }
      hs.leaf.push_back(lf);
      expand_box(box, lb, nullptr);
      hs.bvhLeaves++;
      hs.bvhPrims += lf.count;
      if (depth > hs.bvhDepth) hs.bvhDepth = depth;
      return ~(int32_t)(hs.leaf.size() - 1);
    }
    hs.bvhInternal++;
    int split = (int)(.5 * sz);
    int ax = -1;
    double maxSpan = -1;
    size_t n = lists[0].size();
    for (int i = 0; i < 3; ++i) {  // getIDXofMaxBVHSpan: strict >, ties -> lower axis
      double diff = comp(lists[i][n - 1], i) - comp(lists[i][0], i);
      if (maxSpan < diff) { maxSpan = diff; ax = i; }
    }
    if (ax < 0) ax = 0;
    L lsub(lists[ax].begin(), lists[ax].begin() + split), rsub(lists[ax].begin() + split, lists[ax].begin() + sz);
    L ll[3], rl[3];
    for (int i = 0; i < 3; ++i) {
      if (i == ax) { ll[i] = lsub; rl[i] = rsub; }
      else { sorted(lsub, i, ll[i]); sorted(rsub, i, rl[i]); }
    }
    int me = (int)hs.node.size();
    hs.node.push_back(NodeD());
    Box lb, rbx;
    int32_t lc = bvh(ll, st, st + split, depth + 1, accInv, accXf, lb);
    int32_t rc = bvh(rl, st + split, en, depth + 1, accInv, accXf, rbx);
    NodeD& nd = hs.node[me];
    std::memset(&nd, 0, sizeof(nd));
    for (int c = 0; c < 3; ++c) {
      nd.lmin[c] = lb.mn[c]; nd.lmax[c] = lb.mx[c];
      nd.rmin[c] = rbx.mn[c]; nd.rmax[c] = rbx.mx[c];
    }
    nd.left = lc;
    nd.right = rc;
    expand_box(box, lb, nullptr);
    expand_box(box, rbx, nullptr);
    return me;
  }

  bool build_accel(int ai) {
    const rt_accel_desc& a = d->accels[ai];
    Mat g = ctm_of(a.ctm);
    Mat inv = inverse(g);
    int axf = xf_id(g);
    AccelD ad;
    std::memset(&ad, 0, sizeof(ad));
    ad.xf = axf;
    ad.is_list = (a.type == 0);
    std::vector<int> mem;
    for (int k = 0; k < a.count; ++k) {
      int id = obj_id(d->accel_members[a.first + k]);
      if (id < 0) { err = "accel member out of range"; return false; }
      if (id >= d->num_prims) {
        if (instUsed[id - d->num_prims]++) { err = "instance listed twice"; return false; }
        if (!instance_box(id, ai)) return false;
        accHasInst[ai] = 1;
      }
      mem.push_back(id);
      set_xfc(id, xf_id(mul(g, ctm_of(obj_ctm(id)))));  // reBuildCTMara(objCTM, accelCTM)
    }
    Box box;
    if (a.type == 0) {  // myGeomList: one leaf in insertion order, its own box
      LeafD lf;
      lf.start = (int)hs.member.size();
      lf.count = (int)mem.size();
      for (int p : mem) {
        Mat tmp = mul(inv, ctm_of(obj_ctm(p)));
        expand_box(box, objBox[p], &tmp);
        hs.member.push_back(ref[p]);
      }
      hs.leaf.push_back(lf);
      ad.root = ~(int32_t)(hs.leaf.size() - 1);
    } else {
      L l[3];
      for (int i = 0; i < 3; ++i) sorted(mem, i, l[i]);  // buildSortedObjAras(tmpObjList, -1)
      ad.root = bvh(l, 0, (int)mem.size() - 1, 0, inv, axf, box);
    }
    for (int c = 0; c < 3; ++c) { ad.bmin[c] = box.mn[c]; ad.bmax[c] = box.mx[c]; }
    hs.accel.push_back(ad);
    return true;
  }

  bool run() {
    int n = d->num_prims;
    const int ni = d->num_instances;
    if (ni < 0 || (ni > 0 && !d->instances)) { err = "bad instance list"; return false; }
    ref.assign(n + ni, 0);
    transOrigin.assign(n + ni, d3(0, 0, 0));
    objBox.assign(n + ni, Box());
    boxReady.assign(n + ni, 1);
    for (int j = 0; j < ni; ++j) boxReady[n + j] = 0;
    accHasInst.assign(d->num_accels, 0);
    instUsed.assign(ni, 0);
    hs.nprims = n;
    for (int i = 0; i < n; ++i) {
      if (d->prims[i].material < 0 || d->prims[i].material >= d->num_materials) { err = "bad material index"; return false; }
      if (!build_prim(i)) return false;
    }
    for (int j = 0; j < ni; ++j)
      if (!build_instance(j)) return false;
    for (int a = 0; a < d->num_accels; ++a)
      if (!build_accel(a)) return false;
    if (hs.bvhDepth > 40) { err = "BVH deeper than the kernel traversal stack (40)"; return false; }
    for (int k = 0; k < d->num_top; ++k) {
      int32_t t = d->top[k];
      TopD td;
      std::memset(&td, 0, sizeof(td));
      if (t >= 0 && (t & RT_REF_INSTANCE)) {
        int id = obj_id(t);
        if (id < 0) { err = "top instance out of range"; return false; }
        if (instUsed[id - n]++) { err = "instance listed twice"; return false; }
        const PrimD& q = hs.prim[~ref[id]];
        if ((q.flags & PF_INST_ACCEL) && accHasInst[q.pad[0]]) {
          err = "instance of an accel holding instances is unsupported";
          return false;
        }
        td.kind = TOP_INST;
        td.idx = ~ref[id];
        td.xf = q.xf;
        td.key = q.key;
      } else if (t >= 0) {
        if (t >= n) { err = "top object out of range"; return false; }
        int32_t r = ref[t];
        td.kind = r >= 0 ? TOP_TRI : TOP_PRIM;
        td.idx = r >= 0 ? r : ~r;
        td.xf = r >= 0 ? hs.tri[r].xf : hs.prim[~r].xf;
        td.key = (uint32_t)t;
      } else {
        int ai = ~t;
        if (ai >= d->num_accels) { err = "top accel out of range"; return false; }
        if (d->accels[ai].count == 0) continue;  // empty list/BVH can never report a hit
        td.kind = TOP_ACCEL;
        td.idx = ai;
        td.xf = hs.accel[ai].xf;
      }
      hs.top.push_back(td);
    }
    // materials (myObjShader.setCurrColors, myObjShader.java:51-75)
    for (int m = 0; m < d->num_materials; ++m) {
      const rt_material_desc& s = d->materials[m];
      MatD md;
      std::memset(&md, 0, sizeof(md));
      for (int c = 0; c < 3; ++c) {
        md.diffuse[c] = s.diffuse[c]; md.ambient[c] = s.ambient[c]; md.specular[c] = s.specular[c];
        md.kreflclr[c] = s.k_refl_clr[c]; md.permclr[c] = s.perm_clr[c]; md.periodMult[c] = s.period_mult[c];
      }
      md.avgDiffClr = (1.0 / 3.0) * (s.diffuse[0] + s.diffuse[1] + s.diffuse[2]);
      if (md.avgDiffClr != 0)
        for (int c = 0; c < 3; ++c) md.phtnDiffScl[c] = s.diffuse[c] / md.avgDiffClr;
      double avgPerm = (1.0 / 3.0) * (s.perm_clr[0] + s.perm_clr[1] + s.perm_clr[2]);
      if (avgPerm != 0)
        for (int c = 0; c < 3; ++c) md.phtnPermClr[c] = s.perm_clr[c] / avgPerm;
      md.phong = s.phong_exp; md.krefl = s.k_refl; md.ktrans = s.k_trans; md.perm = s.perm;
      md.diffConst = 1 - s.perm;
      md.hasCaustic = ((s.k_refl > 0.0) || (s.perm > 0.0) || (s.k_trans > 0.0));
      md.simple = s.simple; md.usePhotonMap = s.use_photon_map; md.isCausticPhtn = s.caustic_photons;
      md.tex = s.texture; md.texTop = s.tex_top;
      if (md.tex == RT_TEX_IMAGE && (md.texTop < -1 || md.texTop >= d->num_textures)) { err = "bad texture index"; return false; }
      md.scale = s.noise_scale; md.turbMult = s.turb_mult; md.colorScale = s.color_scale; md.colorMult = s.color_mult;
      md.pmMag = std::sqrt(((s.period_mult[0] * s.period_mult[0]) + (s.period_mult[1] * s.period_mult[1])) +
                           (s.period_mult[2] * s.period_mult[2]));
      md.octaves = s.octaves; md.rndColors = s.rnd_colors; md.useFwdTrans = s.use_fwd_trans;
      if (md.tex >= RT_TEX_NOISE && md.tex <= RT_TEX_WOOD2) {
        if (s.num_colors < 2 || s.num_colors > RT_MAX_NOISE_COLORS) { err = "bad noise colour count"; return false; }
        md.ncolors = s.num_colors;
        for (int k = 0; k < s.num_colors; ++k)
          for (int c = 0; c < 3; ++c) md.colors[k][c] = s.colors[k][c];
      }
      if (md.tex == RT_TEX_STONE) {  // myCellularTexture ctor (myTextureHandler.java:390-425)
        if (s.num_pts_dist > 8) { err = "stone: more than 8 ROI points unsupported"; return false; }
        if (s.num_colors < 4) { err = "stone: needs at least 4 noise colours (mortar pair + a brick pair)"; return false; }
        md.distFunc = s.dist_func; md.roiFunc = s.roi_func; md.numPtsDist = s.num_pts_dist; md.mortar = s.mortar_thresh;
        std::map<double, int> pdfs;  // ConcurrentSkipListMap: put replaces the value of an equal key
        double lastDist = 1.0 / std::pow(M_E, s.avg_per_cell), cumProb = lastDist;
        for (int i = 1; i < 15; ++i) {
          lastDist *= (s.avg_per_cell / (1.0 * i));
          cumProb += lastDist;
          pdfs[cumProb] = i;
        }
        md.npdf = 0;
        for (auto& e : pdfs) { md.pdfKey[md.npdf] = e.first; md.pdfVal[md.npdf] = e.second; md.npdf++; }
      }
      hs.mat.push_back(md);
    }
    // lights (myLight.java:20-30, spot :150-157, disk :244-247)
    for (int l = 0; l < d->num_lights; ++l) {
      const rt_light_desc& s = d->lights[l];
      LightD ld;
      std::memset(&ld, 0, sizeof(ld));
      ld.type = s.type;
      ld.index = l;
      for (int c = 0; c < 3; ++c) { ld.origin[c] = s.pos[c]; ld.color[c] = s.color[c]; }
      D3 o = normalized(d3(s.dir[0], s.dir[1], s.dir[2]));
      ld.orient[0] = o.x; ld.orient[1] = o.y; ld.orient[2] = o.z;
      if (s.type != RT_LIGHT_POINT) {
        D3 t = ortho(o);
        ld.tangent[0] = t.x; ld.tangent[1] = t.y; ld.tangent[2] = t.z;
      }
      ld.innerRad = s.inner_deg * DEG_TO_RAD_F;
      ld.outerRad = s.outer_deg * DEG_TO_RAD_F;
      ld.radDiff = ld.outerRad - ld.innerRad;
      ld.radius = s.radius;
      std::memcpy(ld.g, s.ctm, sizeof(ld.g));
      {  // pad[0] = 1: a point / spot light at its object-space origin (identity CTM): every shadow
         // ray ends there (the device's wave-level shadow cull, trace_kernels.h step_cands)
        bool ident = true;
        for (int q = 0; q < 16; ++q) ident = ident && ld.g[q] == ((q % 5 == 0) ? 1.0 : 0.0);
        ld.pad[0] = (ident && (s.type == RT_LIGHT_POINT || s.type == RT_LIGHT_SPOT)) ? 1 : 0;
      }
      hs.light.push_back(ld);
    }
    // textures -> Processing pixel ints
    int64_t off = 0;
    for (int t = 0; t < d->num_textures; ++t) {
      const rt_texture_desc& s = d->textures[t];
      if (s.w <= 0 || s.h <= 0 || !s.rgb) { err = "bad texture"; return false; }
      TexD td;
      td.w = s.w; td.h = s.h; td.off = off;
      hs.tex.push_back(td);
      for (int64_t k = 0; k < (int64_t)s.w * s.h; ++k)
        hs.texel.push_back(0xFF000000u | ((uint32_t)s.rgb[3 * k] << 16) | ((uint32_t)s.rgb[3 * k + 1] << 8) | s.rgb[3 * k + 2]);
      off += (int64_t)s.w * s.h;
    }
    if (d->bkg_texture >= d->num_textures) { err = "bad background texture"; return false; }
    hs.fov = d->fov;
    for (int c = 0; c < 3; ++c) hs.bg[c] = d->background[c];
    hs.bkgTex = d->bkg_texture;
    for (int c = 0; c < 4; ++c) hs.sky[c] = d->skydome[c];
    hs.dof = d->dof; hs.lensRadius = d->lens_radius; hs.lensFocal = d->lens_focal;
    if (d->camera < RT_CAMERA_FOV || d->camera > RT_CAMERA_ORTHO) { err = "bad camera type"; return false; }
    hs.camera = d->camera;
    hs.cameraParam[0] = d->camera_param[0]; hs.cameraParam[1] = d->camera_param[1];
    if (hs.camera != RT_CAMERA_FOV) hs.dof = 0;  // only myFOVScene.draw uses the lens
    hs.rpp = d->rays_per_pixel;
    hs.photonMode = d->photon_mode; hs.photonCount = d->photon_count; hs.photonK = d->photon_k;
    hs.photonMaxD2 = d->photon_max_dist * d->photon_max_dist;
    return true;
  }
};

// Renumber triangles in leaf order so that a leaf whose members are all triangles holds
// a consecutive run; such a leaf is then encoded in its parent's child reference
// (LEAF_RUN, rt_types.h) and the kernel reads no LeafD and no member index for it --
// two dependent loads fewer per leaf visit. Visit order and all results are unchanged.
void pack_leaves(HostScene& hs) {
  const int nt = (int)hs.tri.size();
  std::vector<int32_t> perm(nt, -1);  // old -> new
  std::vector<int32_t> order;         // new -> old
  order.reserve(nt);
  for (const LeafD& lf : hs.leaf)
    for (int i = 0; i < lf.count; ++i) {
      int32_t r = hs.member[lf.start + i];
      if (r >= 0 && perm[r] < 0) { perm[r] = (int32_t)order.size(); order.push_back(r); }
    }
  for (int r = 0; r < nt; ++r)
    if (perm[r] < 0) { perm[r] = (int32_t)order.size(); order.push_back(r); }
  std::vector<TriD> tri(nt);
  std::vector<double> uv(hs.triUV.size());
  for (int k = 0; k < nt; ++k) {
    tri[k] = hs.tri[order[k]];
    if (!uv.empty()) std::memcpy(&uv[6 * (size_t)k], &hs.triUV[6 * (size_t)order[k]], 6 * sizeof(double));
  }
  hs.tri.swap(tri);
  hs.triUV.swap(uv);
  for (int32_t& r : hs.member)
    if (r >= 0) r = perm[r];
  for (TopD& t : hs.top)
    if (t.kind == TOP_TRI) t.idx = perm[t.idx];
  for (PrimD& q : hs.prim)  // instanced triangles
    if (q.type == PT_INST && !(q.flags & PF_INST_ACCEL) && q.pad[0] >= 0) q.pad[0] = perm[q.pad[0]];
  // child references of leaves that are consecutive triangle runs
  auto code = [&](int32_t child) -> int32_t {
    if (child >= 0) return child;
    const LeafD& lf = hs.leaf[~child];
    if (lf.count <= 0 || lf.count > LEAF_RUN_MAXCOUNT) return child;
    int32_t s0 = hs.member[lf.start];
    if (s0 < 0 || s0 > LEAF_RUN_MAXSTART) return child;
    for (int i = 1; i < lf.count; ++i)
      if (hs.member[lf.start + i] != s0 + i) return child;
    return leaf_run_ref(s0, lf.count);
  };
  for (NodeD& n : hs.node) { n.left = code(n.left); n.right = code(n.right); }
  for (AccelD& a : hs.accel) a.root = code(a.root);
}

// How far outside its edges the reference's triangle test accepts a point (checkInside,
// myPlanarObject.java:165-175: an edge cross product dotted with the unit normal >= -1e-7, i.e.
// 1e-7 / |edge| from the edge line): the corners of that enlarged triangle move by at most
// (d_a + d_b) / sin A. +inf when an angle is too acute to bound (trace.hip tri_world_box, the
// same bound in world space).
static double tri_slack(const TriD& T) {
  double e[3][3], len[3];
  for (int i = 0; i < 3; ++i) {
    for (int c = 0; c < 3; ++c) e[i][c] = T.v[(i + 1) % 3][c] - T.v[i][c];
    len[i] = std::sqrt(e[i][0] * e[i][0] + e[i][1] * e[i][1] + e[i][2] * e[i][2]);
    if (!(len[i] > 0) || !std::isfinite(len[i])) return INFINITY;
  }
  double grow = 0;
  for (int i = 0; i < 3; ++i) {
    const int ia = (i + 2) % 3;
    const double cosA = -(e[ia][0] * e[i][0] + e[ia][1] * e[i][1] + e[ia][2] * e[i][2]) / (len[ia] * len[i]);
    const double sinA = std::sqrt(std::max(0.0, 1 - cosA * cosA));
    if (!(sinA > 1e-4)) return INFINITY;
    const double da = 1e-7 / len[ia] * 1.01 + 1e-12, db = 1e-7 / len[i] * 1.01 + 1e-12;
    grow = std::max(grow, (da + db) / sinA);
  }
  return grow;
}

// Fat-edge bounds of every node child of the accels that qualify for the nearest-first
// closest-hit traversal (AccelD.flags): a BVH whose leaves are all triangle runs in the
// accel's own CTM. A child's bound is its triangles' largest tri_slack plus a relative
// 2^-30 of its box coordinates (the hit point's own rounding; generous on purpose).
static void nearest_first_bounds(HostScene& hs) {
  for (AccelD& a : hs.accel) {
    a.flags = 0;
    if (a.is_list || a.root < 0) continue;
    bool ok = true;
    std::vector<int32_t> stack{a.root};
    std::vector<int32_t> order;  // nodes, parents first
    while (!stack.empty() && ok) {
      const int32_t r = stack.back();
      stack.pop_back();
      order.push_back(r);
      for (int side = 0; side < 2; ++side) {
        const int32_t c = side ? hs.node[r].right : hs.node[r].left;
        if (c >= 0) { stack.push_back(c); continue; }
        if (!((~c) & LEAF_RUN_FLAG)) { ok = false; break; }  // a LeafD leaf (prims / instances)
        const int32_t st = ((~c) >> 5) & LEAF_RUN_MAXSTART, cnt = (~c) & 31;
        for (int i = 0; i < cnt; ++i)
          if (hs.tri[st + i].xf != a.xf) { ok = false; break; }
      }
    }
    if (!ok) continue;
    std::vector<double> sub(hs.node.size(), 0.0);  // a node's largest slack over its subtree
    for (auto it = order.rbegin(); it != order.rend() && ok; ++it) {
      NodeD& n = hs.node[*it];
      double m = 0;
      for (int side = 0; side < 2; ++side) {
        const int32_t c = side ? n.right : n.left;
        double s = 0;
        if (c >= 0) s = sub[c];
        else {
          const int32_t st = ((~c) >> 5) & LEAF_RUN_MAXSTART, cnt = (~c) & 31;
          for (int i = 0; i < cnt; ++i) s = std::max(s, tri_slack(hs.tri[st + i]));
        }
        if (!std::isfinite(s)) { ok = false; break; }
        const double* mn = side ? n.rmin : n.lmin;
        const double* mx = side ? n.rmax : n.lmax;
        double mag = 0;
        for (int k = 0; k < 3; ++k) mag = std::max(mag, std::max(std::fabs(mn[k]), std::fabs(mx[k])));
        node_slack(n, side) = s * 1.01 + mag * 0x1p-30 + 1e-300;
        m = std::max(m, s);
      }
      sub[*it] = m;
    }
    if (ok) a.flags |= ACCEL_NEAREST;
  }
}

}  // namespace

int build_host_scene(const rt_scene_desc* d, HostScene& hs) {
  Builder b(d, hs);
  if (!b.run()) return set_error(RT_E_INVALID, b.err);
  if (hs.leaf.size() >= (size_t)LEAF_RUN_FLAG) return set_error(RT_E_INVALID, "too many BVH leaves");
  pack_leaves(hs);
  nearest_first_bounds(hs);
  return RT_OK;
}

}  // namespace rt
