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

}  // namespace

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
}

}  // namespace rt
