// Photon-map search structure (host). The reference stores photon_list in a
// one-photon-per-node kd-tree (myKD_Tree.build_tree, myLight.java:325-381) and
// answers getIrradianceFromPhtnTree (myObjShader.java:441-458) with the k nearest
// photons within max_dist. That set is a property of the photon list, not of the
// tree, so the device uses a structure that suits 64-wide waves: a BVH whose leaves
// are ranges of <= PHOTON_LEAF photons stored contiguously (positions / powers as
// double[3] in leaf order) -- a query walks ~log2(n/24) nodes and scans whole
// leaves instead of chasing one dependent pointer per photon.
//
// Build: median partition of the photon index range on the axis of largest extent
// (order by (coordinate, index)), boxes from the photons' exact coordinates; a leaf's
// photons in id order. photon_build.hip builds the same structure on the GPU (the
// default for maps above one leaf); this host build stays for tiny maps and as the
// reference the device build is tested against (DISTRAYTRACER_PHOTON_BUILD=host).
#include <algorithm>
#include <cstring>
#include <thread>
#include <utility>

#include "rt_internal.h"

namespace rt {
namespace {

struct PhotonBvh {
  const std::vector<double>& pos;
  std::vector<int>& idx;
  std::vector<NodeD>& nodes;
  std::vector<std::pair<int, int>> leaves;  // leaf ranges [lo, hi)

  void box(int lo, int hi, double* mn, double* mx) const {
    for (int c = 0; c < 3; ++c) { mn[c] = 1e300; mx[c] = -1e300; }
    for (int i = lo; i < hi; ++i) {
      const double* q = &pos[3 * (size_t)idx[i]];
      for (int c = 0; c < 3; ++c) {
        mn[c] = std::min(mn[c], q[c]);
        mx[c] = std::max(mx[c], q[c]);
      }
    }
  }
  // Subtree over idx[lo, hi) as a child of its parent: a node index (>= 0), or -1 for a
  // leaf whose range the parent keeps in NodeD.pad (left: pad[0..1], right: pad[2], padR[0]).
  int32_t build(int lo, int hi, bool force_node = false) {
    if (hi - lo <= PHOTON_LEAF && !force_node) {
      leaves.emplace_back(lo, hi);
      return -1;
    }
    double mn[3], mx[3];
    box(lo, hi, mn, mx);
    int ax = 0;
    for (int c = 1; c < 3; ++c)
      if (mx[c] - mn[c] > mx[ax] - mn[ax]) ax = c;
    const int mid = (hi - lo <= PHOTON_LEAF) ? hi : lo + (hi - lo) / 2;  // tiny maps: one leaf + an empty one
    if (mid < hi)  // median partition on (coordinate, photon index): deterministic
      std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, [&](int a, int b) {
        const double va = pos[3 * (size_t)a + ax], vb = pos[3 * (size_t)b + ax];
        return va < vb || (va == vb && a < b);
      });
    const int me = (int)nodes.size();
    nodes.push_back(NodeD());
    const int32_t l = build(lo, mid);
    const int32_t r = build(mid, hi);
    NodeD& nd = nodes[me];
    std::memset(&nd, 0, sizeof(nd));
    box(lo, mid, nd.lmin, nd.lmax);
    box(mid, hi, nd.rmin, nd.rmax);
    nd.left = l;
    nd.right = r;
    nd.pad[0] = lo; nd.pad[1] = mid - lo;
    nd.pad[2] = mid; nd.padR[0] = hi - mid;
    nd.padR[1] = hi - lo;  // photons in the subtree
    return me;
  }
};

// myKD_Tree.build_tree (myLight.java:332-381) over photon_list indices: a range of one photon is a
// leaf; otherwise the axis of largest extent (mins / maxs from +-1e20, `dx >= dy && dx >= dz` -> x,
// then y, then z), Collections.sort of the range on that coordinate -- stable, `<` / `>` compares,
// so the previous order breaks ties and -0 ties +0 -- and the median at size / 2 becomes the node.
// A range of m photons holds exactly m nodes, numbered in DFS pre-order: the left child of node q
// is q + 1, the right one q + 1 + split. Subtrees near the root are built on their own threads.
struct JavaKd {
  const double* pos;
  int32_t* idx;
  KdNodeD* out;
  void sort_range(int lo, int hi, int ax, std::vector<int32_t>& buf) const {
    const int n = hi - lo;
    int32_t* a = idx + lo;
    auto key = [&](int32_t i) { return pos[3 * (size_t)i + ax]; };
    if (n <= 24) {  // stable insertion sort
      for (int i = 1; i < n; ++i) {
        const int32_t v = a[i];
        const double kv = key(v);
        int j = i - 1;
        while (j >= 0 && kv < key(a[j])) { a[j + 1] = a[j]; --j; }
        a[j + 1] = v;
      }
      return;
    }
    // stable merge sort with a caller-owned buffer (no allocation per node)
    buf.resize(n);
    for (int w = 1; w < n; w *= 2) {
      for (int l = 0; l < n; l += 2 * w) {
        const int m = std::min(l + w, n), r = std::min(l + 2 * w, n);
        int i = l, j = m, o = l;
        while (i < m && j < r) buf[o++] = (key(a[j]) < key(a[i])) ? a[j++] : a[i++];
        while (i < m) buf[o++] = a[i++];
        while (j < r) buf[o++] = a[j++];
      }
      std::copy(buf.begin(), buf.begin() + n, a);
    }
  }
  void build(int lo, int hi, int q, int depth) {
    std::vector<int32_t> buf;
    build_(lo, hi, q, depth, buf);
  }
  void build_(int lo, int hi, int q, int depth, std::vector<int32_t>& buf) {
    const int n = hi - lo;
    if (n == 1) {
      out[q] = KdNodeD{idx[lo], -1, -1, -1};
      return;
    }
    double mn[3] = {1e20, 1e20, 1e20}, mx[3] = {-1e20, -1e20, -1e20};
    for (int i = lo; i < hi; ++i) {
      const double* p = pos + 3 * (size_t)idx[i];
      for (int c = 0; c < 3; ++c) {
        if (p[c] < mn[c]) mn[c] = p[c];
        if (p[c] > mx[c]) mx[c] = p[c];
      }
    }
    const double dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
    const int ax = (dx >= dy && dx >= dz) ? 0 : (dy >= dx && dy >= dz) ? 1 : 2;
    sort_range(lo, hi, ax, buf);
    const int split = n / 2;
    const int qr = q + 1 + split;
    out[q] = KdNodeD{idx[lo + split], ax, split != 0 ? q + 1 : -1, split != n - 1 ? qr : -1};
    if (depth < 4 && n > 4096) {  // the two subtrees in parallel
      std::thread t([this, lo, split, q, depth] { if (split != 0) build(lo, lo + split, q + 1, depth + 1); });
      if (split != n - 1) build_(lo + split + 1, hi, qr, depth + 1, buf);
      t.join();
    } else {
      if (split != 0) build_(lo, lo + split, q + 1, depth + 1, buf);
      if (split != n - 1) build_(lo + split + 1, hi, qr, depth + 1, buf);
    }
  }
};

}  // namespace

std::vector<KdNodeD> build_java_kdtree(const std::vector<double>& pos) {
  const int n = (int)(pos.size() / 3);
  std::vector<KdNodeD> out(n);
  if (n == 0) return out;
  std::vector<int32_t> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  JavaKd b{pos.data(), idx.data(), out.data()};
  b.build(0, n, 0, 0);
  return out;
}

void kd_to_leaf_order(std::vector<KdNodeD>& kd, const std::vector<int32_t>& leafToList) {
  std::vector<int32_t> leafOf(leafToList.size());
  for (size_t i = 0; i < leafToList.size(); ++i) leafOf[leafToList[i]] = (int32_t)i;
  for (KdNodeD& k : kd) k.photon = leafOf[k.photon];
}

void build_photon_tree(HostScene& hs, const std::vector<double>& pos, const std::vector<double>& pwr) {
  hs.photonListPos = pos;
  hs.photonListPwr = pwr;
  hs.pnode.clear();
  hs.ppos.clear();
  hs.ppwr.clear();
  const int n = (int)(pos.size() / 3);
  hs.nphoton = n;
  hs.photonRoot = 0;
  hs.pnodeCount = 0;
  if (n == 0) return;
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  PhotonBvh b{pos, idx, hs.pnode, {}};
  hs.photonRoot = b.build(0, n, true);  // the root is always a node
  hs.pnodeCount = (int64_t)hs.pnode.size();
  // photons of a leaf in id order (deterministic; the same as the device build, photon_build.hip)
  for (auto& lf : b.leaves) std::sort(idx.begin() + lf.first, idx.begin() + lf.second);
  hs.ppos.resize(3 * (size_t)n);
  hs.ppwr.resize(3 * (size_t)n);
  for (int i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      hs.ppos[3 * (size_t)i + c] = pos[3 * (size_t)idx[i] + c];
      hs.ppwr[3 * (size_t)i + c] = pwr[3 * (size_t)idx[i] + c];
    }
  // the reference's kd-tree after the BVH records (KdNodeD), photons as leaf-order indices
  std::vector<KdNodeD> kd = build_java_kdtree(pos);
  kd_to_leaf_order(kd, idx);
  const size_t off = hs.pnode.size();
  hs.pnode.resize(off + (kd.size() + KD_PER_NODED - 1) / KD_PER_NODED);
  std::memcpy(&hs.pnode[off], kd.data(), kd.size() * sizeof(KdNodeD));
  hs.pnode[hs.photonRoot].padR[2] = (int32_t)off;
}

}  // namespace rt

// Host-only: the reference's kd-tree over a photon_list (photon = list index), for tests.
extern "C" int rt_photon_kdtree(const double* pos, int64_t n, int32_t* out) {
  if (n < 0 || (n > 0 && (!pos || !out))) return rt::set_error(RT_E_INVALID, "rt_photon_kdtree: bad arguments");
  if (n > INT32_MAX / 4) return rt::set_error(RT_E_INVALID, "rt_photon_kdtree: too many photons");
  std::vector<double> p(pos, pos + 3 * n);
  std::vector<rt::KdNodeD> kd = rt::build_java_kdtree(p);
  std::memcpy(out, kd.data(), kd.size() * sizeof(rt::KdNodeD));
  return RT_OK;
}
