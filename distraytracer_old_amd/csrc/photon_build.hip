// GPU build of the photon-map search structure: the same median BVH as the host builder
// (csrc/photon.cpp, which documents the structure), level by level on the device.
//
// The host recursion splits each photon range [lo, hi) (> PHOTON_LEAF photons, or the root)
// at mid = lo + (hi - lo) / 2 on the axis of largest extent, the left half being the
// (mid - lo) smallest photons in (coordinate, photon index) order. Here:
//  * three lists hold the photon ids sorted by (x, id), (y, id), (z, id) -- one stable
//    radix sort each, the key being the coordinate + 0.0 (so -0 == +0, as the host's
//    comparator treats them);
//  * every list stays sorted within each range, so a range's box is read from the first
//    and last entries of the three lists, and its left half is the first (mid - lo)
//    entries of the split axis' list;
//  * one level = all ranges of one depth: flag the left halves, then stably partition each
//    list within its ranges (an exclusive scan of the flags gives every entry's place).
// Node numbering is the host's DFS pre-order: the number of internal nodes under a range
// depends on its photon count only (T(c) = 0 for c <= PHOTON_LEAF, else 1 + T(c/2) +
// T(c - c/2)), so a right child is numbered parent + 1 + T(left count). Leaf photons are
// ordered by photon id (as the host's leaves are), so both builders produce the same
// nodes, boxes and leaf-ordered photon arrays: images are bit-identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>
#include <map>

#include "rt_internal.h"

namespace rt {
namespace pb {

struct Range {
  int32_t lo, cnt;
  int32_t parent;  // node whose child this range is (-1: the root)
  int32_t side;    // 0 left, 1 right
  int32_t node;    // this range's node (DFS pre-order), -1 when it is a leaf
  int32_t axis, mid, pad;
};

static constexpr int TMAX = 128;
struct TTable {  // T(c) for the <= 2 counts per level
  int32_t n;
  int32_t c[TMAX];
  int32_t t[TMAX];
};

__device__ inline int32_t t_of(const TTable& T, int32_t c) {
  if (c <= PHOTON_LEAF) return 0;
  for (int i = 0; i < T.n; ++i)
    if (T.c[i] == c) return T.t[i];
  return -1;  // not reached: the host tabulates every count of the tree
}

__global__ void k_keys(const double* __restrict__ pos, int32_t n, int c, double* __restrict__ key,
                       int32_t* __restrict__ id) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  key[i] = pos[3 * (size_t)i + c] + 0.0;
  id[i] = i;
}

// One thread per range: its box (from the sorted lists) and reference go into its parent;
// an internal range also fills its own node's ranges and picks its split.
__global__ void k_ranges(const double* __restrict__ pos, const int32_t* __restrict__ L0, const int32_t* __restrict__ L1,
                         const int32_t* __restrict__ L2, Range* __restrict__ rg, int32_t nr, NodeD* __restrict__ nodes,
                         int32_t* __restrict__ internal, int32_t* __restrict__ leafStart) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  Range R = rg[r];
  const int32_t* L[3] = {L0, L1, L2};
  double mn[3], mx[3];
  for (int c = 0; c < 3; ++c) {
    mn[c] = pos[3 * (size_t)L[c][R.lo] + c];
    mx[c] = pos[3 * (size_t)L[c][R.lo + R.cnt - 1] + c];
  }
  if (R.parent >= 0) {
    NodeD& P = nodes[R.parent];
    double* bmn = R.side ? P.rmin : P.lmin;
    double* bmx = R.side ? P.rmax : P.lmax;
    for (int c = 0; c < 3; ++c) { bmn[c] = mn[c]; bmx[c] = mx[c]; }
    if (R.side) P.right = R.node;
    else P.left = R.node;
  }
  internal[r] = R.node >= 0;
  if (R.node < 0) {
    leafStart[R.lo] = R.cnt;
    return;
  }
  int ax = 0;
  for (int c = 1; c < 3; ++c)
    if (mx[c] - mn[c] > mx[ax] - mn[ax]) ax = c;
  const int32_t mid = R.lo + R.cnt / 2;
  NodeD& N = nodes[R.node];
  N.pad[0] = R.lo; N.pad[1] = mid - R.lo;
  N.pad[2] = mid; N.padR[0] = R.lo + R.cnt - mid;
  N.padR[1] = R.cnt;
  N.padR[2] = 0;
  rg[r].axis = ax;
  rg[r].mid = mid;
}

// the two children of every internal range, in range order (so the next level stays sorted by lo)
__global__ void k_children(const Range* __restrict__ rg, int32_t nr, const int32_t* __restrict__ base,
                           Range* __restrict__ next, TTable T) {
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  const Range R = rg[r];
  if (R.node < 0) return;
  const int32_t lc = R.mid - R.lo, rc = R.cnt - lc;
  Range a{R.lo, lc, R.node, 0, lc > PHOTON_LEAF ? R.node + 1 : -1, 0, 0, 0};
  Range b{R.mid, rc, R.node, 1, rc > PHOTON_LEAF ? R.node + 1 + t_of(T, lc) : -1, 0, 0, 0};
  next[2 * base[r]] = a;
  next[2 * base[r] + 1] = b;
}

// range of list position p at this level (-1: p lies in a leaf finished earlier)
__device__ inline int32_t range_of(const Range* rg, int32_t nr, int32_t p) {
  int32_t a = 0, b = nr - 1;
  while (a < b) {  // last range with lo <= p
    const int32_t m = (a + b + 1) >> 1;
    if (rg[m].lo <= p) a = m;
    else b = m - 1;
  }
  const Range& R = rg[a];
  return (R.lo <= p && p < R.lo + R.cnt && R.node >= 0) ? a : -1;
}

__global__ void k_locate(const Range* __restrict__ rg, int32_t nr, int32_t n, int32_t* __restrict__ posRange) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  posRange[p] = range_of(rg, nr, p);
}

// left[id] for the photons of internal ranges: the first (mid - lo) entries of the split axis' list
__global__ void k_mark(const Range* __restrict__ rg, const int32_t* __restrict__ posRange, int32_t n,
                       const int32_t* __restrict__ L0, const int32_t* __restrict__ L1, const int32_t* __restrict__ L2,
                       uint8_t* __restrict__ left) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t r = posRange[p];
  if (r < 0) return;
  const Range& R = rg[r];
  const int32_t* L = R.axis == 0 ? L0 : (R.axis == 1 ? L1 : L2);
  left[L[p]] = p < R.mid;
}

__global__ void k_flags(const int32_t* __restrict__ posRange, int32_t n, const int32_t* __restrict__ L,
                        const uint8_t* __restrict__ left, int32_t* __restrict__ f) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  f[p] = posRange[p] >= 0 ? left[L[p]] : 0;
}

// stable partition of one list within every internal range (scan = exclusive sum of the flags)
__global__ void k_scatter(const Range* __restrict__ rg, const int32_t* __restrict__ posRange, int32_t n,
                          const int32_t* __restrict__ L, const int32_t* __restrict__ scan, const int32_t* __restrict__ f,
                          int32_t* __restrict__ out) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t r = posRange[p];
  int32_t q = p;
  if (r >= 0) {
    const Range& R = rg[r];
    const int32_t before = scan[p] - scan[R.lo];  // left entries of this range before p
    q = f[p] ? R.lo + before : R.mid + (p - R.lo) - before;
  }
  out[q] = L[p];
}

// leaves: photons ordered by id; then the leaf-ordered position / power arrays
__global__ void k_leaf_order(const int32_t* __restrict__ leafStart, int32_t n, int32_t* __restrict__ L) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int32_t c = leafStart[p];
  for (int32_t i = p + 1; i < p + c; ++i) {  // insertion sort of <= PHOTON_LEAF ids
    const int32_t v = L[i];
    int32_t j = i - 1;
    while (j >= p && L[j] > v) { L[j + 1] = L[j]; --j; }
    L[j + 1] = v;
  }
}

__global__ void k_gather(const int32_t* __restrict__ L, int32_t n, const double* __restrict__ pos,
                         const double* __restrict__ pwr, double* __restrict__ ppos, double* __restrict__ ppwr) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const size_t s = 3 * (size_t)L[p], d = 3 * (size_t)p;
  for (int c = 0; c < 3; ++c) { ppos[d + c] = pos[s + c]; ppwr[d + c] = pwr[s + c]; }
}

// internal nodes of the median tree over c photons (the root of a map is always a node)
static int64_t t_count(int64_t c, std::map<int64_t, int64_t>& memo) {
  if (c <= PHOTON_LEAF) return 0;
  auto it = memo.find(c);
  if (it != memo.end()) return it->second;
  const int64_t v = 1 + t_count(c / 2, memo) + t_count(c - c / 2, memo);
  memo[c] = v;
  return v;
}

// ---------------------------------------------------------------------------
// The reference's kd-tree (myKD_Tree.build_tree, myLight.java:332-381; KdNodeD) on the device, level
// by level. Every range ("segment") of a level holds its photons in the reference's current order,
// contiguously, in segment order. One level: the segments' extents (wave-aggregated 64-bit atomic
// min / max of order-preserving keys; mins / maxs start from +-1e20 like the Java) pick each split
// axis; two stable radix sorts -- every photon by its coordinate on its segment's axis (+ 0.0: -0
// ties +0 as Java's `<` does), then by segment -- are Collections.sort of every segment at once (a
// tie keeps the previous order); the median at size / 2 becomes the node, the two sides the next
// level's segments (a side of one photon is a leaf at once). Nodes are numbered in DFS pre-order:
// the left child of node q is q + 1, the right one q + 1 + split.
namespace kd {
struct Seg {
  int32_t start, size, node, axis;
  int32_t lid, rid, lstart, rstart;  // the children's next-level segments (-1: none) and positions
};
__device__ inline uint64_t okey(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v + 0.0);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double okey_inv(uint64_t k) {
  return __builtin_bit_cast(double, (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k);
}
__global__ void k_iota(int32_t* __restrict__ perm, int32_t* __restrict__ segOf, int32_t n) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { perm[i] = i; segOf[i] = 0; }
}
__global__ void k_ext_init(unsigned long long* __restrict__ ext, int32_t nseg) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nseg * 6) ext[i] = (i % 6) < 3 ? ~0ull : 0ull;
}
// 64-thread blocks: a wave whose photons are all in one segment reduces first (one atomic per value)
__global__ void __launch_bounds__(64) k_ext(const double* __restrict__ pos, const int32_t* __restrict__ perm,
                                            const int32_t* __restrict__ segOf, int32_t nAct, unsigned long long* __restrict__ ext) {
  const int32_t p = blockIdx.x * 64 + threadIdx.x;
  const bool valid = p < nAct;
  const int32_t s = valid ? segOf[p] : -1;
  unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0, 0, 0};
  if (valid)
    for (int c = 0; c < 3; ++c) mn[c] = mx[c] = okey(pos[3 * (size_t)perm[p] + c]);
  const int32_t s0 = __shfl(s, 0);
  if (__all(!valid || s == s0)) {
    for (int off = 32; off >= 1; off >>= 1)
      for (int c = 0; c < 3; ++c) {
        const unsigned long long a = __shfl_xor(mn[c], off), b = __shfl_xor(mx[c], off);
        mn[c] = a < mn[c] ? a : mn[c];
        mx[c] = b > mx[c] ? b : mx[c];
      }
    if (threadIdx.x == 0)
      for (int c = 0; c < 3; ++c) { atomicMin(ext + 6 * s0 + c, mn[c]); atomicMax(ext + 6 * s0 + 3 + c, mx[c]); }
  } else if (valid) {
    for (int c = 0; c < 3; ++c) { atomicMin(ext + 6 * s + c, mn[c]); atomicMax(ext + 6 * s + 3 + c, mx[c]); }
  }
}
__global__ void k_axis(Seg* __restrict__ seg, const unsigned long long* __restrict__ ext, int32_t nseg) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  double d[3];
  for (int c = 0; c < 3; ++c) {  // mins / maxs from +-1e20 (build_tree :343-353)
    const double lo = fmin(1e20, okey_inv(ext[6 * i + c])), hi = fmax(-1e20, okey_inv(ext[6 * i + 3 + c]));
    d[c] = hi - lo;
  }
  seg[i].axis = (d[0] >= d[1] && d[0] >= d[2]) ? 0 : (d[1] >= d[0] && d[1] >= d[2]) ? 1 : 2;
}
__global__ void k_keys(const double* __restrict__ pos, const int32_t* __restrict__ perm, const int32_t* __restrict__ segOf,
                       const Seg* __restrict__ seg, int32_t nAct, uint64_t* __restrict__ key, uint64_t* __restrict__ val) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nAct) return;
  const int32_t s = segOf[p], i = perm[p];
  key[p] = okey(pos[3 * (size_t)i + seg[s].axis]);
  val[p] = ((uint64_t)(uint32_t)s << 32) | (uint32_t)i;
}
__global__ void k_unpack(const uint64_t* __restrict__ val, int32_t nAct, uint32_t* __restrict__ skey, int32_t* __restrict__ perm) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nAct) return;
  skey[p] = (uint32_t)(val[p] >> 32);
  perm[p] = (int32_t)(uint32_t)val[p];
}
__global__ void k_seg_count(const Seg* __restrict__ seg, int32_t nseg, int32_t* __restrict__ emits, int32_t* __restrict__ elems) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  const int32_t split = seg[i].size / 2, nl = split, nr = seg[i].size - split - 1;
  emits[i] = (nl > 1) + (nr > 1);
  elems[i] = (nl > 1 ? nl : 0) + (nr > 1 ? nr : 0);
}
__global__ void k_seg_make(Seg* __restrict__ seg, int32_t nseg, const int32_t* __restrict__ perm,
                           const int32_t* __restrict__ leafOf, const int32_t* __restrict__ sbase, const int32_t* __restrict__ pbase,
                           KdNodeD* __restrict__ kd, Seg* __restrict__ next) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  Seg S = seg[i];
  const int32_t split = S.size / 2, nl = split, nr = S.size - split - 1;
  const int32_t q = S.node, ql = q + 1, qr = q + 1 + split;
  kd[q] = KdNodeD{leafOf[perm[S.start + split]], S.axis, nl > 0 ? ql : -1, nr > 0 ? qr : -1};
  if (nl == 1) kd[ql] = KdNodeD{leafOf[perm[S.start]], -1, -1, -1};
  if (nr == 1) kd[qr] = KdNodeD{leafOf[perm[S.start + split + 1]], -1, -1, -1};
  int32_t b = sbase[i], pb = pbase[i];
  S.lid = S.rid = -1;
  if (nl > 1) { S.lid = b; S.lstart = pb; next[b] = Seg{pb, nl, ql, 0, -1, -1, 0, 0}; ++b; pb += nl; }
  if (nr > 1) { S.rid = b; S.rstart = pb; next[b] = Seg{pb, nr, qr, 0, -1, -1, 0, 0}; }
  seg[i] = S;
}
__global__ void k_move(const Seg* __restrict__ seg, const uint32_t* __restrict__ skey, const int32_t* __restrict__ perm,
                       int32_t nAct, int32_t* __restrict__ perm2, int32_t* __restrict__ segOf2) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nAct) return;
  const Seg& S = seg[skey[p]];
  const int32_t j = p - S.start, split = S.size / 2;
  if (j < split && S.lid >= 0) { perm2[S.lstart + j] = perm[p]; segOf2[S.lstart + j] = S.lid; }
  else if (j > split && S.rid >= 0) { perm2[S.rstart + (j - split - 1)] = perm[p]; segOf2[S.rstart + (j - split - 1)] = S.rid; }
}
__global__ void k_leaf_of(const int32_t* __restrict__ L0, int32_t n, int32_t* __restrict__ leafOf) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) leafOf[L0[i]] = i;
}
}  // namespace kd

struct DevBuf {  // scratch allocations of one build, freed on every path
  std::vector<void*> p;
  template <class T>
  hipError_t alloc(T** out, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) p.push_back(q);
    *out = (T*)q;
    return e;
  }
  ~DevBuf() {
    for (void* q : p) (void)hipFree(q);
  }
};

}  // namespace pb

#define PBCHK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) return set_error(RT_E_HIP, std::string("photon map build: ") + hipGetErrorString(e_)); \
  } while (0)

// Build the photon map of photon_list (pos / pwr, insertion order) on the scene's device.
// out: device arrays owned by the scene (allocs); n > PHOTON_LEAF.
// the reference's kd-tree of photon_list (device pos, list order) into kdOut, photons as leaf-order
// indices (leafOf[list index])
static int build_java_kdtree_gpu(const double* pos, int32_t n, const int32_t* leafOf, KdNodeD* kdOut) {
  using namespace pb;
  using namespace pb::kd;
  const int TB = 256;
  auto grid = [&](int64_t m) { return dim3((unsigned)std::max<int64_t>(1, (m + TB - 1) / TB)); };
  DevBuf tmp;
  int32_t *perm, *perm2, *segOf, *segOf2, *emits, *elems, *sbase, *pbase;
  uint32_t *skey, *skey2;
  uint64_t *key, *key2, *val, *val2;
  unsigned long long* ext;
  Seg *seg, *next;
  const size_t maxSeg = (size_t)n / 2 + 2;
  PBCHK(tmp.alloc(&perm, n)); PBCHK(tmp.alloc(&perm2, n));
  PBCHK(tmp.alloc(&segOf, n)); PBCHK(tmp.alloc(&segOf2, n));
  PBCHK(tmp.alloc(&skey, n)); PBCHK(tmp.alloc(&skey2, n));
  PBCHK(tmp.alloc(&key, n)); PBCHK(tmp.alloc(&key2, n));
  PBCHK(tmp.alloc(&val, n)); PBCHK(tmp.alloc(&val2, n));
  PBCHK(tmp.alloc(&ext, 6 * maxSeg));
  PBCHK(tmp.alloc(&seg, maxSeg)); PBCHK(tmp.alloc(&next, maxSeg));
  PBCHK(tmp.alloc(&emits, maxSeg)); PBCHK(tmp.alloc(&elems, maxSeg));
  PBCHK(tmp.alloc(&sbase, maxSeg)); PBCHK(tmp.alloc(&pbase, maxSeg));
  size_t b1 = 0, b2 = 0, b3 = 0;
  PBCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, key, key2, val, val2, n));
  PBCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, skey, skey2, perm, perm2, n));
  PBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, b3, emits, sbase, (int)maxSeg));
  void* cub = nullptr;
  const size_t cb = std::max(b1, std::max(b2, b3));
  PBCHK(tmp.alloc((char**)&cub, cb));
  hipLaunchKernelGGL(k_iota, grid(n), dim3(TB), 0, 0, perm, segOf, n);
  const Seg root{0, n, 0, 0, -1, -1, 0, 0};
  PBCHK(hipMemcpy(seg, &root, sizeof(Seg), hipMemcpyHostToDevice));
  int32_t nseg = 1, nAct = n;
  while (nseg > 0) {
    int segBits = 1;
    while ((1ll << segBits) < nseg) ++segBits;
    hipLaunchKernelGGL(k_ext_init, grid(6LL * nseg), dim3(TB), 0, 0, ext, nseg);
    hipLaunchKernelGGL(k_ext, dim3((unsigned)((nAct + 63) / 64)), dim3(64), 0, 0, pos, perm, segOf, nAct, ext);
    hipLaunchKernelGGL(k_axis, grid(nseg), dim3(TB), 0, 0, seg, ext, nseg);
    hipLaunchKernelGGL(k_keys, grid(nAct), dim3(TB), 0, 0, pos, perm, segOf, seg, nAct, key, val);
    PBCHK(hipGetLastError());
    size_t b = cb;  // the coordinate on the segment's axis, then the segment: stable, so ties keep the order
    PBCHK(hipcub::DeviceRadixSort::SortPairs(cub, b, key, key2, val, val2, nAct));
    hipLaunchKernelGGL(k_unpack, grid(nAct), dim3(TB), 0, 0, val2, nAct, skey, perm);
    b = cb;
    PBCHK(hipcub::DeviceRadixSort::SortPairs(cub, b, skey, skey2, perm, perm2, nAct, 0, segBits));
    hipLaunchKernelGGL(k_seg_count, grid(nseg), dim3(TB), 0, 0, seg, nseg, emits, elems);
    b = cb;
    PBCHK(hipcub::DeviceScan::ExclusiveSum(cub, b, emits, sbase, nseg));
    b = cb;
    PBCHK(hipcub::DeviceScan::ExclusiveSum(cub, b, elems, pbase, nseg));
    hipLaunchKernelGGL(k_seg_make, grid(nseg), dim3(TB), 0, 0, seg, nseg, perm2, leafOf, sbase, pbase, kdOut, next);
    hipLaunchKernelGGL(k_move, grid(nAct), dim3(TB), 0, 0, seg, skey2, perm2, nAct, perm, segOf);
    PBCHK(hipGetLastError());
    int32_t lastS[2], lastE[2];
    PBCHK(hipMemcpy(lastS, sbase + nseg - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    PBCHK(hipMemcpy(lastS + 1, emits + nseg - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    PBCHK(hipMemcpy(lastE, pbase + nseg - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    PBCHK(hipMemcpy(lastE + 1, elems + nseg - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    nseg = lastS[0] + lastS[1];
    nAct = lastE[0] + lastE[1];
    std::swap(seg, next);
  }
  PBCHK(hipDeviceSynchronize());
  return RT_OK;
}

int build_photon_tree_gpu(rt_scene* s, const double* pos_h, const double* pwr_h, int64_t n64) {
  using namespace pb;
  const int32_t n = (int32_t)n64;
  const int TB = 256;
  const unsigned gn = (unsigned)((n + TB - 1) / TB);
  std::map<int64_t, int64_t> memo;
  const int64_t nnodes = t_count(n, memo);
  TTable T{};
  for (auto& kv : memo) {
    if (T.n >= TMAX) return set_error(RT_E_INVALID, "photon map build: count table overflow");
    T.c[T.n] = (int32_t)kv.first;
    T.t[T.n] = (int32_t)kv.second;
    ++T.n;
  }
  DevBuf tmp;
  double *pos, *pwr, *key, *keyAlt;
  int32_t *id, *L[3], *Lalt, *posRange, *f, *scan, *leafStart, *internal, *base;
  uint8_t* left;
  Range *rg, *next;
  const size_t maxRanges = (size_t)n / (PHOTON_LEAF / 2) + 4;
  PBCHK(tmp.alloc(&pos, 3 * (size_t)n));
  PBCHK(tmp.alloc(&pwr, 3 * (size_t)n));
  PBCHK(tmp.alloc(&key, n));
  PBCHK(tmp.alloc(&keyAlt, n));
  PBCHK(tmp.alloc(&id, n));
  for (int c = 0; c < 3; ++c) PBCHK(tmp.alloc(&L[c], n));
  PBCHK(tmp.alloc(&Lalt, n));
  PBCHK(tmp.alloc(&posRange, n));
  PBCHK(tmp.alloc(&f, n));
  PBCHK(tmp.alloc(&scan, n));
  PBCHK(tmp.alloc(&leafStart, n));
  PBCHK(tmp.alloc(&left, n));
  PBCHK(tmp.alloc(&rg, maxRanges));
  PBCHK(tmp.alloc(&next, maxRanges));
  PBCHK(tmp.alloc(&internal, maxRanges));
  PBCHK(tmp.alloc(&base, maxRanges));
  // results (scene-owned)
  NodeD* nodes = nullptr;
  double *ppos = nullptr, *ppwr = nullptr;
  const int64_t kdRecs = (n64 + KD_PER_NODED - 1) / KD_PER_NODED;  // the reference's kd-tree after the BVH
  PBCHK(hipMalloc(&nodes, sizeof(NodeD) * (nnodes + kdRecs)));
  s->allocs.push_back(nodes);
  PBCHK(hipMalloc(&ppos, sizeof(double) * 3 * (size_t)n));
  s->allocs.push_back(ppos);
  PBCHK(hipMalloc(&ppwr, sizeof(double) * 3 * (size_t)n));
  s->allocs.push_back(ppwr);
  s->devBytes += sizeof(NodeD) * (nnodes + kdRecs) + 2 * sizeof(double) * 3 * (size_t)n;
  PBCHK(hipMemset(nodes, 0, sizeof(NodeD) * (nnodes + kdRecs)));
  PBCHK(hipMemset(leafStart, 0, sizeof(int32_t) * n));
  PBCHK(hipMemcpy(pos, pos_h, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice));
  PBCHK(hipMemcpy(pwr, pwr_h, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice));
  // scratch of the library primitives (sized for the largest call)
  size_t sortBytes = 0, scanBytes = 0, scanBytesR = 0;
  PBCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, sortBytes, key, keyAlt, id, L[0], n));
  PBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scanBytes, f, scan, n));
  PBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scanBytesR, internal, base, (int)maxRanges));
  void* cub = nullptr;
  PBCHK(tmp.alloc((char**)&cub, std::max(sortBytes, std::max(scanBytes, scanBytesR))));
  // the three (coordinate, id) orders
  for (int c = 0; c < 3; ++c) {
    hipLaunchKernelGGL(k_keys, dim3(gn), dim3(TB), 0, 0, pos, n, c, key, id);
    PBCHK(hipGetLastError());
    size_t b = sortBytes;
    PBCHK(hipcub::DeviceRadixSort::SortPairs(cub, b, key, keyAlt, id, L[c], n));
  }
  // level by level
  Range root{0, n, -1, 0, 0, 0, 0, 0};
  PBCHK(hipMemcpy(rg, &root, sizeof(Range), hipMemcpyHostToDevice));
  int32_t nr = 1;
  while (nr > 0) {
    const unsigned gr = (unsigned)((nr + TB - 1) / TB);
    hipLaunchKernelGGL(k_ranges, dim3(gr), dim3(TB), 0, 0, pos, L[0], L[1], L[2], rg, nr, nodes, internal, leafStart);
    PBCHK(hipGetLastError());
    size_t b = scanBytesR;
    PBCHK(hipcub::DeviceScan::ExclusiveSum(cub, b, internal, base, nr));
    int32_t lastBase = 0, lastInt = 0;
    PBCHK(hipMemcpy(&lastBase, base + nr - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    PBCHK(hipMemcpy(&lastInt, internal + nr - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    const int32_t nint = lastBase + lastInt;
    if (nint == 0) break;
    if ((size_t)2 * nint > maxRanges) return set_error(RT_E_INVALID, "photon map build: range overflow");
    hipLaunchKernelGGL(k_children, dim3(gr), dim3(TB), 0, 0, rg, nr, base, next, T);
    hipLaunchKernelGGL(k_locate, dim3(gn), dim3(TB), 0, 0, rg, nr, n, posRange);
    hipLaunchKernelGGL(k_mark, dim3(gn), dim3(TB), 0, 0, rg, posRange, n, L[0], L[1], L[2], left);
    PBCHK(hipGetLastError());
    for (int c = 0; c < 3; ++c) {
      hipLaunchKernelGGL(k_flags, dim3(gn), dim3(TB), 0, 0, posRange, n, L[c], left, f);
      size_t bs = scanBytes;
      PBCHK(hipcub::DeviceScan::ExclusiveSum(cub, bs, f, scan, n));
      hipLaunchKernelGGL(k_scatter, dim3(gn), dim3(TB), 0, 0, rg, posRange, n, L[c], scan, f, Lalt);
      PBCHK(hipGetLastError());
      std::swap(L[c], Lalt);
    }
    std::swap(rg, next);
    nr = 2 * nint;
  }
  hipLaunchKernelGGL(k_leaf_order, dim3(gn), dim3(TB), 0, 0, leafStart, n, L[0]);
  hipLaunchKernelGGL(k_gather, dim3(gn), dim3(TB), 0, 0, L[0], n, pos, pwr, ppos, ppwr);
  PBCHK(hipGetLastError());
  PBCHK(hipDeviceSynchronize());
  {  // the reference's kd-tree after the BVH records, photons as leaf-order indices
    int32_t* leafOf = nullptr;
    PBCHK(tmp.alloc(&leafOf, n));
    hipLaunchKernelGGL(pb::kd::k_leaf_of, dim3(gn), dim3(TB), 0, 0, L[0], n, leafOf);
    PBCHK(hipGetLastError());
    int rc = build_java_kdtree_gpu(pos, n, leafOf, reinterpret_cast<KdNodeD*>(nodes + nnodes));
    if (rc) return rc;
    const int32_t off = (int32_t)nnodes;
    PBCHK(hipMemcpy(&nodes[0].padR[2], &off, sizeof(int32_t), hipMemcpyHostToDevice));
  }
  s->dev.pnode = nodes;
  s->dev.ppos = ppos;
  s->dev.ppwr = ppwr;
  s->dev.nphoton = n;
  s->dev.photonRoot = 0;
  s->hs.pnode.clear();
  s->hs.ppos.clear();
  s->hs.ppwr.clear();
  s->hs.photonRoot = 0;
  s->hs.nphoton = n;
  s->hs.pnodeCount = nnodes;
  s->photonsUploaded = true;
  return RT_OK;
}

}  // namespace rt
