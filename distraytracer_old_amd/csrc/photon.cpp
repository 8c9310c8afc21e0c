// Photon kd-tree build on the host (myKD_Tree.build_tree, myLight.java:325-381):
// split axis = largest extent (ties x, then y, z), Collections.sort (stable) on
// that axis, median = size/2 stored at the node, children [0,split) and
// (split, size). Input order = the reference's photon_list insertion order.
#include <algorithm>
#include <utility>

#include "rt_internal.h"

namespace rt {
namespace {

struct KdBuilder {
  const std::vector<double>& pos;
  const std::vector<double>& pwr;
  std::vector<PhotonD>& nodes;
  std::vector<std::pair<double, int>> tmp;

  int build(std::vector<int>& idx, int lo, int hi) {
    int sz = hi - lo;
    PhotonD n;
    std::memset(&n, 0, sizeof(n));
    if (sz == 1) {
      int p = idx[lo];
      for (int c = 0; c < 3; ++c) { n.pos[c] = pos[3 * p + c]; n.pwr[c] = pwr[3 * p + c]; }
      n.axis = -1; n.left = n.right = -1;
      nodes.push_back(n);
      return (int)nodes.size() - 1;
    }
    double mins[3] = {1e20, 1e20, 1e20}, maxs[3] = {-1e20, -1e20, -1e20};
    for (int i = lo; i < hi; i++) {
      const double* q = &pos[3 * idx[i]];
      for (int j = 0; j < 3; j++) {
        if (q[j] < mins[j]) mins[j] = q[j];
        if (q[j] > maxs[j]) maxs[j] = q[j];
      }
    }
    double dx = maxs[0] - mins[0], dy = maxs[1] - mins[1], dz = maxs[2] - mins[2];
    int ax = 2;
    if (dx >= dy && dx >= dz) ax = 0;
    else if (dy >= dx && dy >= dz) ax = 1;
    tmp.resize(sz);
    for (int i = 0; i < sz; ++i) tmp[i] = std::make_pair(pos[3 * idx[lo + i] + ax], idx[lo + i]);
    std::stable_sort(tmp.begin(), tmp.end(), [](const std::pair<double, int>& a, const std::pair<double, int>& b) {
      return a.first < b.first;
    });
    for (int i = 0; i < sz; ++i) idx[lo + i] = tmp[i].second;
    int split = sz / 2;
    int p = idx[lo + split];
    for (int c = 0; c < 3; ++c) { n.pos[c] = pos[3 * p + c]; n.pwr[c] = pwr[3 * p + c]; }
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
};

}  // namespace

void build_photon_tree(HostScene& hs, const std::vector<double>& pos, const std::vector<double>& pwr) {
  hs.photon.clear();
  hs.photonRoot = -1;
  int n = (int)(pos.size() / 3);
  if (n == 0) return;
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  hs.photon.reserve(n);
  KdBuilder b{pos, pwr, hs.photon, {}};
  hs.photonRoot = b.build(idx, 0, n);
}

}  // namespace rt
