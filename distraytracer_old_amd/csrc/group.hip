// Multi-GPU frame behind the C ABI (include/distraytracer.h rt_group_*).
//
// The reference renders one image on one thread (myFOVScene.draw, myScene.java:1481-1531); pixels
// and their samples are independent, so the frame shards by wave tiles. A group is N ranks, one GPU
// each (or N ranks sharing devices for the one-GPU emulation), each holding the replicated scene:
//
//   plan     rank 0's measured wave time of every tile of the whole-frame layout (rt_tile_costs)
//            cut into N contiguous runs of equal cost; tiles whose own wave would outlast a rank's
//            share are rendered one sample per wave beside the run (plan_ranks, deterministic, so
//            every process derives the same plan from the broadcast costs);
//   step     rank r renders its run (tile list) + split pixels into a whole-frame buffer on its
//            stream; ranks r > 0 pack their pixels (pack_kernel) and send them to rank 0 over RCCL
//            (ncclSend / ncclRecv in one group: each rank's pixels cross its own xGMI link into rank
//            0 once) or, in the one-process emulation, by device copies; rank 0, which rendered its
//            own run straight into the output frame, scatters the received pixels into it
//            (scatter_kernel). The exchange runs on a third stream per rank with double-buffered
//            send / receive slabs, so frame f's exchange overlaps frame f + 1's render.
//
// Pixels, their RNG keys and their per-pixel sample order do not depend on the plan, so the frame
// equals the 1-GPU frame bit for bit for every N and transport.
//
// Transports: RCCL (one device per rank; in one process ncclCommInitAll, one process per GPU an
// rt_comm from rt_comm_create_rccl), the host transport of an rt_comm made by rt_comm_create_host
// (caller callbacks on pinned host staging; ranks may share a device, so the rank-mode path runs as
// N processes on one GPU), or device copies in one process (RT_GROUP_COPY, the one-GPU emulation).
// In rank mode every collective carries the ranks' status so that all ranks fail together, and
// every cut of the plan ends in a plan check: each sender's offset, pixel count and pixel-list hash
// against the receive side rank 0 derives (plan_check).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "comm.h"

using namespace rt;

#define GCHK(expr)                                                                       \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return set_error(RT_E_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------------------------------------
// plan (host only; multigpu.py rank_plans is the independent Python restatement the tests compare)
namespace rt {
// owner[t]: rank in [0, world) rendering tile t in its wave run, or world + rank when the tile is
// one of that rank's split (one sample per wave) tiles. order: every tile in dispatch order --
// longest first by quarter-octave cost bucket, row-major inside a bucket; a rank's run and split
// tiles are the subsequences of `order` it owns.
void plan_ranks(const uint32_t* cost, int n, int world, double heavy, int slots, int32_t* owner, int32_t* order,
                const double* weight) {
  // contiguous cut: tile t goes to the rank holding its cost midpoint (prefix sums of integer costs,
  // exact in double for < 2^53). weight (rt_group_rebalance, may be null): the cut runs over
  // cost x weight instead -- the ranks' measured speed folded into their tiles' costs
  double total = 0;
  for (int t = 0; t < n; ++t) total += (double)cost[t];
  double wtotal = total;
  if (weight) {
    wtotal = 0;
    for (int t = 0; t < n; ++t) wtotal += (double)cost[t] * weight[t];
  }
  double cum = 0;
  for (int t = 0; t < n; ++t) {
    const double c = weight ? (double)cost[t] * weight[t] : (double)cost[t];
    cum += c;
    int r;
    if (wtotal > 0) {
      const double mid = cum - 0.5 * c;
      const double q = (mid * world) / wtotal;
      r = (int)std::min<int64_t>((int64_t)q, world - 1);
    } else {
      r = (int)((int64_t)t * world / std::max(1, n));
    }
    owner[t] = r;
  }
  // heavy tiles: a wave longer than `heavy` x a rank's ideal per-slot share is split per sample
  // (from the measured wave times themselves: whether a wave outlasts a share does not depend on
  // the rank it lands on)
  if (world > 1) {
    const double thr = heavy * total / ((double)slots * world);
    for (int t = 0; t < n; ++t)
      if ((double)cost[t] > thr) owner[t] += world;
  }
  // dispatch order: counting sort by bucket, longest first, stable (row-major inside a bucket)
  constexpr int NB = 4 * 32 + 1;
  std::vector<int> start(NB, 0);
  std::vector<uint8_t> key(n);
  for (int t = 0; t < n; ++t) {
    key[t] = (uint8_t)cost_bucket(cost[t]);
    start[key[t]]++;
  }
  for (int k = NB - 1, acc = 0; k >= 0; --k) {
    const int h = start[k];
    start[k] = acc;
    acc += h;
  }
  for (int t = 0; t < n; ++t) order[start[key[t]]++] = t;
}
}  // namespace rt

// ---------------------------------------------------------------------------------------------
// pack / scatter kernels (ARGB int32 and the optional float-RGB plane)
__global__ void __launch_bounds__(256) pack_kernel(const int32_t* __restrict__ argb, const float* __restrict__ rgb,
                                                   const int32_t* __restrict__ idx, int n, int32_t* __restrict__ oa,
                                                   float* __restrict__ orgb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t p = idx[i];
  oa[i] = argb[p];
  if (orgb) {
    orgb[3 * (int64_t)i + 0] = rgb[3 * p + 0];
    orgb[3 * (int64_t)i + 1] = rgb[3 * p + 1];
    orgb[3 * (int64_t)i + 2] = rgb[3 * p + 2];
  }
}
__global__ void __launch_bounds__(256) scatter_kernel(const int32_t* __restrict__ ia, const float* __restrict__ irgb,
                                                      const int32_t* __restrict__ idx, int n, int32_t* __restrict__ argb,
                                                      float* __restrict__ rgb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t p = idx[i];
  argb[p] = ia[i];
  if (rgb) {
    rgb[3 * p + 0] = irgb[3 * (int64_t)i + 0];
    rgb[3 * p + 1] = irgb[3 * (int64_t)i + 1];
    rgb[3 * p + 2] = irgb[3 * (int64_t)i + 2];
  }
}

// ---------------------------------------------------------------------------------------------
namespace {
constexpr int KRING = 64;  // frames of kernel-time events kept per rank

struct GRank {
  rt_scene* s = nullptr;
  int dev = 0, rank = 0;
  hipStream_t st = nullptr, side = nullptr, cs = nullptr;  // render, split pixels, exchange
  ParamsD P{};
  std::vector<int32_t> hTiles, hSplit, hPix, hAll;  // run tiles, split tiles, split pixels, every pixel written
  int32_t *dTiles = nullptr, *dPix = nullptr, *dAll = nullptr;
  double* smpCol = nullptr;
  uint8_t* smpTr = nullptr;
  float* fRgb[2] = {};  // whole-frame render targets of frames f and f + 1 (ranks > 0): frame f's pack (on
  int32_t* fArgb[2] = {};  // the exchange stream) reads one while frame f + 1 renders into the other
  float* sRgb[2] = {};
  int32_t* sArgb[2] = {};
  hipEvent_t evStart = nullptr, evSide = nullptr, evSent[2] = {}, evRendered = nullptr;
  hipEvent_t evFree[2] = {};  // render target b read by its pack (the render of frame f + 2 may start)
  hipEvent_t tA[KRING] = {}, tB[KRING] = {};
  int64_t timed = 0;  // frames with kernel events since the last rt_group_kernel_ms
  ncclComm_t nccl = nullptr;  // RCCL transport: this rank's communicator (rank mode: the rt_comm's, borrowed)
  int64_t off = 0;  // offset of this rank's pixels in rank 0's receive slab
};
}  // namespace

struct rt_group {
  int world = 1;
  bool rankMode = false, useRccl = false, rgb = false, root = false;
  bool hostX = false;        // rank mode over a host-transport rt_comm: the exchange staged through pinned memory
  rt_comm* comm = nullptr;   // rank mode at world > 1 (owned when ownComm: rt_group_create_rank)
  bool ownComm = false;
  int64_t planChecks = 0;    // collective plan checks passed (plan_check)
  std::vector<uint64_t> pixHash;  // per rank: hash of the pixel list it sends (rank_lists `all`)
  char* hSend = nullptr;     // host transport: pinned staging of this rank's packed pixels / rank 0's slab
  char* hRecv = nullptr;
  uint32_t renderFlags = 0;
  rt_render_params p{};
  int W = 0, H = 0, ntiles = 0, tilesX = 0, tw = 0, th = 0;
  std::vector<int32_t> owner, order;
  std::vector<uint32_t> cost;  // the layout's measured wave times (the plan's input)
  std::vector<double> weight;  // per-tile cut weights (rt_group_rebalance; empty: none)
  double heavy = 1.25;
  int slots = 4096;
  std::vector<int64_t> npix;   // pixels written per rank
  std::vector<GRank> r;        // the ranks this process drives (all of them in local mode)
  // rank 0 (root) state
  int rootDev = 0;
  int64_t nRecv = 0;
  int32_t* dScat = nullptr;     // pixels of ranks 1.. in receive-slab order
  float* rRgb[2] = {};
  int32_t* rArgb[2] = {};
  float* outRgb = nullptr;      // internal frame (rt_group_render with NULL outputs, rt_group_render_host)
  int32_t* outArgb = nullptr;
  void* stage = nullptr;        // pinned read-back staging (rt_group_render_host)
  hipEvent_t evRecv[2] = {};    // receive slab b consumed by its scatter
  std::vector<hipEvent_t> evCopied;  // COPY transport: rank r's copy into the slab done
  int64_t frame = 0;
  std::vector<void*> allocs;      // for the group's life (streams' frames, rank 0's output)
  std::vector<void*> planAllocs;  // per plan (setup_lists; freed when rt_group_rebalance re-cuts)
  std::vector<void*> planHost;    // per plan, pinned host (hSend / hRecv)
};

namespace {
int gmalloc(rt_group* g, void** p, size_t bytes, bool plan = false) {
  *p = nullptr;
  if (bytes == 0) return RT_OK;
  GCHK(hipMalloc(p, bytes));
  (plan ? g->planAllocs : g->allocs).push_back(*p);
  return RT_OK;
}
template <class T>
int gupload(rt_group* g, const std::vector<T>& v, T** out) {  // a plan's list
  int rc = gmalloc(g, (void**)out, v.size() * sizeof(T), true);
  if (rc || v.empty()) return rc;
  GCHK(hipMemcpy(*out, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return RT_OK;
}

// pixels (row * W + col) of tile t of the whole-frame layout, row-major inside the tile, clipped
void tile_pixels(const rt_group* g, int t, std::vector<int32_t>& out) {
  const int tx = t % g->tilesX, ty = t / g->tilesX;
  for (int dy = 0; dy < g->th; ++dy)
    for (int dx = 0; dx < g->tw; ++dx) {
      const int row = ty * g->th + dy, col = tx * g->tw + dx;
      if (row < g->H && col < g->W) out.push_back(row * g->W + col);
    }
}

// host lists of rank q from the plan
void rank_lists(const rt_group* g, int q, std::vector<int32_t>& tiles, std::vector<int32_t>& split,
                std::vector<int32_t>& pix, std::vector<int32_t>& all) {
  tiles.clear(); split.clear(); pix.clear(); all.clear();
  for (int t : g->order) {
    if (g->owner[t] == q) tiles.push_back(t);
    else if (g->owner[t] == g->world + q) split.push_back(t);
  }
  for (int t : split) tile_pixels(g, t, pix);
  for (int t : tiles) tile_pixels(g, t, all);
  all.insert(all.end(), pix.begin(), pix.end());
}

int destroy_group(rt_group* g);
int sync_group(rt_group* g);

// once per group: the per-rank streams and events, rank 0's slab events, the whole-frame buffers
int setup_streams(rt_group* g) {
  const size_t npx = (size_t)g->W * g->H;
  for (GRank& R : g->r) {
    GCHK(hipSetDevice(R.dev));
    int rc;
    if ((rc = prepare_render(R.s, &g->p, R.P))) return rc;
    GCHK(hipStreamCreateWithFlags(&R.st, hipStreamNonBlocking));
    GCHK(hipStreamCreateWithFlags(&R.side, hipStreamNonBlocking));
    GCHK(hipStreamCreateWithFlags(&R.cs, hipStreamNonBlocking));
    GCHK(hipEventCreateWithFlags(&R.evStart, hipEventDisableTiming));
    GCHK(hipEventCreateWithFlags(&R.evSide, hipEventDisableTiming));
    GCHK(hipEventCreateWithFlags(&R.evRendered, hipEventDisableTiming));
    for (int b = 0; b < 2; ++b) GCHK(hipEventCreateWithFlags(&R.evFree[b], hipEventDisableTiming));
    for (int b = 0; b < 2; ++b) GCHK(hipEventCreateWithFlags(&R.evSent[b], hipEventDisableTiming));
    for (int k = 0; k < KRING; ++k) {
      GCHK(hipEventCreate(&R.tA[k]));
      GCHK(hipEventCreate(&R.tB[k]));
    }
    if (R.rank != 0) {
      for (int b = 0; b < (g->world > 1 ? 2 : 1); ++b) {
        if ((rc = gmalloc(g, (void**)&R.fArgb[b], npx * sizeof(int32_t)))) return rc;
        if (g->rgb && (rc = gmalloc(g, (void**)&R.fRgb[b], npx * 3 * sizeof(float)))) return rc;
      }
    }
  }
  if (g->root) {
    GCHK(hipSetDevice(g->rootDev));
    int rc;
    for (int b2 = 0; b2 < 2; ++b2) GCHK(hipEventCreateWithFlags(&g->evRecv[b2], hipEventDisableTiming));
    if ((rc = gmalloc(g, (void**)&g->outArgb, npx * sizeof(int32_t)))) return rc;
    if (g->rgb && (rc = gmalloc(g, (void**)&g->outRgb, npx * 3 * sizeof(float)))) return rc;
    if (!g->useRccl) {
      g->evCopied.assign(g->world, nullptr);
      for (int q = 0; q < g->world; ++q) GCHK(hipEventCreateWithFlags(&g->evCopied[q], hipEventDisableTiming));
    }
  }
  return RT_OK;
}

// FNV-1a of a pixel list (plan_check compares the lists the ranks derive without sending them)
uint64_t hash_list(const std::vector<int32_t>& v) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)v.size();
  for (int32_t x : v) {
    h ^= (uint32_t)x;
    h *= 1099511628211ull;
  }
  return h;
}

// rank 0's receive offset of rank q's pixels: the slab holds ranks 1, 2, ... in rank order (the RCCL
// and host receive loops); a sender's own R.off comes from setup_lists, and plan_check compares them
int64_t recv_offset(const rt_group* g, int q) {
  int64_t o = 0;
  for (int k = 1; k < q; ++k) o += g->npix[k];
  return o;
}

// per plan (again after rt_group_rebalance): the ranks' tile / pixel lists on the device, their
// sample buffers and send slabs, rank 0's scatter list and receive slabs (this process's ranks only;
// plan_check makes it collective in rank mode)
int setup_lists_local(rt_group* g) {
  if (!g->planAllocs.empty() || !g->planHost.empty()) {  // a re-cut: the previous plan's buffers, once no stream uses them
    int rc0 = sync_group(g);
    if (rc0) return rc0;
    for (void* p : g->planAllocs) GCHK(hipFree(p));
    for (void* p : g->planHost) GCHK(hipHostFree(p));
    g->planAllocs.clear();
    g->planHost.clear();
    g->hSend = g->hRecv = nullptr;
  }
  g->npix.assign(g->world, 0);
  g->pixHash.assign(g->world, 0);
  {
    std::vector<int32_t> a, b, c, d;
    for (int q = 0; q < g->world; ++q) {
      rank_lists(g, q, a, b, c, d);
      g->npix[q] = (int64_t)d.size();
      g->pixHash[q] = hash_list(d);
    }
  }
  int64_t off = 0;
  std::vector<int64_t> offs(g->world, 0);
  for (int q = 1; q < g->world; ++q) { offs[q] = off; off += g->npix[q]; }
  g->nRecv = off;
  for (GRank& R : g->r) {
    GCHK(hipSetDevice(R.dev));
    int rc;
    rank_lists(g, R.rank, R.hTiles, R.hSplit, R.hPix, R.hAll);
    R.off = offs[R.rank];
    if ((rc = gupload(g, R.hTiles, &R.dTiles)) || (rc = gupload(g, R.hPix, &R.dPix)) || (rc = gupload(g, R.hAll, &R.dAll)))
      return rc;
    const size_t ns = R.hPix.size() * (size_t)R.P.spp;
    if ((rc = gmalloc(g, (void**)&R.smpCol, ns * 3 * sizeof(double), true)) || (rc = gmalloc(g, (void**)&R.smpTr, ns, true))) return rc;
    if (R.rank != 0)
      for (int b = 0; b < 2; ++b) {
        if ((rc = gmalloc(g, (void**)&R.sArgb[b], R.hAll.size() * sizeof(int32_t), true))) return rc;
        if (g->rgb && (rc = gmalloc(g, (void**)&R.sRgb[b], R.hAll.size() * 3 * sizeof(float), true))) return rc;
      }
  }
  if (g->root) {
    GCHK(hipSetDevice(g->rootDev));
    std::vector<int32_t> scat;
    scat.reserve(g->nRecv);
    std::vector<int32_t> a, b, c, d;
    for (int q = 1; q < g->world; ++q) {
      rank_lists(g, q, a, b, c, d);
      scat.insert(scat.end(), d.begin(), d.end());
    }
    int rc;
    if ((rc = gupload(g, scat, &g->dScat))) return rc;
    for (int b2 = 0; b2 < 2; ++b2) {
      if ((rc = gmalloc(g, (void**)&g->rArgb[b2], g->nRecv * sizeof(int32_t), true))) return rc;
      if (g->rgb && (rc = gmalloc(g, (void**)&g->rRgb[b2], g->nRecv * 3 * sizeof(float), true))) return rc;
    }
  }
  if (g->hostX) {  // pinned staging of the host transport: a sender's packed pixels, rank 0's whole slab
    const size_t px = sizeof(int32_t) + (g->rgb ? 3 * sizeof(float) : 0);
    const GRank& R = g->r[0];
    const size_t bytes = R.rank == 0 ? (size_t)g->nRecv * px : R.hAll.size() * px;
    if (bytes) {
      void* h = nullptr;
      GCHK(hipHostMalloc(&h, bytes));
      g->planHost.push_back(h);
      (R.rank == 0 ? g->hRecv : g->hSend) = (char*)h;
    }
  }
  return RT_OK;
}

// Rank mode, world > 1: every rank's {status, rank, offset in rank 0's slab, pixel count, pixel-list
// hash, plan hash} all-gathered and checked by every rank against its own derivation of the plan --
// the receive offsets and counts rank 0's receive loop uses (recv_offset, npix) and the pixel lists
// (pixHash). A rank's local failure or any disagreement fails every rank here, before a frame
// exchange could block on a mismatched send / receive.
int plan_check(rt_group* g, int local_rc) {
  if (!g->rankMode || g->world == 1 || !g->comm) return local_rc;
  const std::string mine = local_rc ? std::string(rt_last_error()) : std::string();
  uint64_t plan = hash_list(g->owner) ^ (hash_list(g->order) * 31);
  const GRank* R = g->r.empty() ? nullptr : &g->r[0];
  const int64_t rec[6] = {local_rc, R ? R->rank : -1, R ? R->off : -1, R ? (int64_t)R->hAll.size() : -1,
                          (int64_t)(local_rc || !R ? 0 : g->pixHash[R->rank]), (int64_t)plan};
  std::vector<int64_t> all(6 * (size_t)g->world);
  int rc = comm_allgather(g->comm, rec, all.data(), sizeof(rec));
  if (rc) return rc;
  if (local_rc) return set_error(local_rc, mine);
  for (int q = 0; q < g->world; ++q) {
    const int64_t* x = &all[6 * (size_t)q];
    if (x[0]) return set_error((int)x[0], "rt_group: rank " + std::to_string(q) + " failed its setup; every rank stops");
    std::string why;
    if (x[1] != q) why = "reports rank " + std::to_string(x[1]);
    else if (x[5] != (int64_t)plan) why = "derived a different plan (owner / order)";
    else if (q > 0 && x[2] != recv_offset(g, q))
      why = "sends at offset " + std::to_string(x[2]) + " of rank 0's slab, rank 0 receives it at " + std::to_string(recv_offset(g, q));
    else if (x[3] != g->npix[q]) why = "sends " + std::to_string(x[3]) + " pixels, rank 0 receives " + std::to_string(g->npix[q]);
    else if (x[4] != (int64_t)g->pixHash[q]) why = "sends a different pixel list";
    if (!why.empty()) return set_error(RT_E_INVALID, "rt_group plan check: rank " + std::to_string(q) + " " + why);
  }
  g->planChecks++;
  return RT_OK;
}

int setup_lists(rt_group* g) { return plan_check(g, setup_lists_local(g)); }

int setup_ranks(rt_group* g) {
  int rc = setup_streams(g);
  if (rc == RT_OK) rc = setup_lists_local(g);
  return plan_check(g, rc);
}

int make_layout(rt_group* g, rt_scene* s, const rt_render_params* p, uint32_t flags) {
  if (!p) return set_error(RT_E_INVALID, "rt_group: null params");
  if (p->flags & (RT_RENDER_WAVEFRONT | RT_RENDER_PIXEL_WAVES))
    return set_error(RT_E_INVALID, "rt_group: RT_RENDER_WAVEFRONT / RT_RENDER_PIXEL_WAVES are not group layouts");
  g->p = *p;
  g->p.row0 = 0; g->p.row1 = p->height; g->p.row_step = 1; g->p.row_band = 1;
  g->p.flags = p->flags & ~(uint32_t)RT_RENDER_ROWMAJOR;
  g->rgb = (flags & RT_GROUP_RGB) != 0;
  g->W = p->width;
  g->H = p->height;
  ParamsD P{};
  int rc = prepare_render(s, &g->p, P);
  if (rc) return rc;
  const int ncols = P.W;
  g->tw = P.tw; g->th = P.th;
  g->tilesX = (ncols + P.tw - 1) / P.tw;
  g->ntiles = g->tilesX * ((P.nrows + P.th - 1) / P.th);
  return RT_OK;
}

int make_plan(rt_group* g, const std::vector<uint32_t>& cost, double heavy, int slots) {
  if (!(heavy > 0)) heavy = 1.25;
  if (slots <= 0) slots = 4096;
  g->cost = cost;
  g->heavy = heavy;
  g->slots = slots;
  g->owner.assign(g->ntiles, 0);
  g->order.assign(g->ntiles, 0);
  plan_ranks(cost.data(), g->ntiles, g->world, heavy, slots, g->owner.data(), g->order.data(),
             g->weight.empty() ? nullptr : g->weight.data());
  return RT_OK;
}

GRank* local_rank(rt_group* g, int rank) {
  for (GRank& R : g->r)
    if (R.rank == rank) return &R;
  return nullptr;
}

// rank R's render of the frame into (rgb, argb) on R.st (split pixels on R.side beside it)
int enqueue_render(rt_group* g, GRank& R, float* rgb, int32_t* argb, bool timed) {
  GCHK(hipSetDevice(R.dev));
  if (timed) GCHK(hipEventRecord(R.tA[R.timed % KRING], R.st));
  int rc;
  if (!R.hPix.empty()) {
    GCHK(hipEventRecord(R.evStart, R.st));
    GCHK(hipStreamWaitEvent(R.side, R.evStart, 0));
    if ((rc = launch_pixel_list(R.s, R.P, g->p.flags, R.dPix, (int)R.hPix.size(), R.smpCol, R.smpTr, rgb, argb, R.side)))
      return rc;
    GCHK(hipEventRecord(R.evSide, R.side));
  }
  if (!R.hTiles.empty() && (rc = launch_tile_list(R.s, R.P, g->p.flags, R.dTiles, (int)R.hTiles.size(), rgb, argb, R.st)))
    return rc;
  if (!R.hPix.empty()) GCHK(hipStreamWaitEvent(R.st, R.evSide, 0));
  if (timed) {
    GCHK(hipEventRecord(R.tB[R.timed % KRING], R.st));
    R.timed++;
  }
  return RT_OK;
}

// rank R (> 0): frame f's render into target b on R.st, after frame f - 2's pack has read it
int enqueue_rank_render(rt_group* g, GRank& R, int b, bool timed) {
  GCHK(hipSetDevice(R.dev));
  GCHK(hipStreamWaitEvent(R.st, R.evFree[b], 0));
  return enqueue_render(g, R, R.fRgb[b], R.fArgb[b], timed);
}

// rank R (> 0): pack its pixels of render target b into send slab b on the exchange stream, once the
// render is done -- off the render stream, so the next frame's render starts at once. The exchange
// stream's own order puts it after the send that last used slab b.
int enqueue_pack(rt_group* g, GRank& R, int b) {
  const int n = (int)R.hAll.size();
  GCHK(hipEventRecord(R.evRendered, R.st));
  GCHK(hipStreamWaitEvent(R.cs, R.evRendered, 0));
  if (n > 0) {
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, R.cs, R.fArgb[b], R.fRgb[b], R.dAll, n,
                       R.sArgb[b], g->rgb ? R.sRgb[b] : nullptr);
    GCHK(hipGetLastError());
  }
  GCHK(hipEventRecord(R.evFree[b], R.cs));
  return RT_OK;
}

// root: scatter receive slab b (pixels [lo, hi) of it) into the frame on stream cs
int enqueue_scatter(rt_group* g, hipStream_t cs, int b, int64_t lo, int64_t hi, float* rgb, int32_t* argb) {
  const int n = (int)(hi - lo);
  if (n <= 0) return RT_OK;
  hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, cs, g->rArgb[b] + lo,
                     g->rgb ? g->rRgb[b] + 3 * lo : nullptr, g->dScat + lo, n, argb, g->rgb ? rgb : nullptr);
  GCHK(hipGetLastError());
  return RT_OK;
}

// one frame; rgb / argb: rank 0's output frame on its device (NULL: the internal frame)
int group_frame(rt_group* g, float* rgb, int32_t* argb) {
  const int b = (int)(g->frame & 1);
  if (g->root) {
    if (!argb) argb = g->outArgb;
    if (!rgb) rgb = g->outRgb;
    if (rgb && !g->rgb) return set_error(RT_E_INVALID, "rt_group: float-RGB output needs RT_GROUP_RGB");
  }
  int rc;
  // renders (+ packs) of every local rank
  for (GRank& R : g->r) {
    if (R.rank == 0) {
      if ((rc = enqueue_render(g, R, rgb, argb, true))) return rc;
    } else if ((rc = enqueue_rank_render(g, R, b, true)) || (rc = enqueue_pack(g, R, b))) {
      return rc;
    }
  }
  GRank* R0 = g->root ? local_rank(g, 0) : nullptr;
  if (g->world > 1) {
    if (g->useRccl) {
      // the single exchange: ranks > 0 send their packed pixels to rank 0 (grouped point-to-point)
      if (R0) {
        GCHK(hipSetDevice(R0->dev));
        GCHK(hipStreamWaitEvent(R0->cs, g->evRecv[b], 0));
      }
      // a failed call inside the group is recorded and the group still closed (an open group
      // would leave every later RCCL call of this thread queued)
      ncclResult_t first = g_rccl.groupStart();
      if (first != ncclSuccess) return set_error(RT_E_HIP, std::string("ncclGroupStart failed: ") + g_rccl.errStr(first));
      auto keep = [&](ncclResult_t r) {
        if (first == ncclSuccess) first = r;
      };
      for (GRank& R : g->r) {
        const size_t n = R.hAll.size();
        if (R.rank != 0 && n) {
          keep(g_rccl.send(R.sArgb[b], n, ncclInt32, 0, R.nccl, R.cs));
          if (g->rgb) keep(g_rccl.send(R.sRgb[b], 3 * n, ncclFloat32, 0, R.nccl, R.cs));
        }
      }
      if (R0)
        for (int q = 1; q < g->world; ++q) {
          const int64_t o = recv_offset(g, q);
          const size_t n = (size_t)g->npix[q];
          if (!n) continue;
          keep(g_rccl.recv(g->rArgb[b] + o, n, ncclInt32, q, R0->nccl, R0->cs));
          if (g->rgb) keep(g_rccl.recv(g->rRgb[b] + 3 * o, 3 * n, ncclFloat32, q, R0->nccl, R0->cs));
        }
      keep(g_rccl.groupEnd());
      if (first != ncclSuccess) return set_error(RT_E_HIP, std::string("RCCL frame exchange failed: ") + g_rccl.errStr(first));
      for (GRank& R : g->r)
        if (R.rank != 0) {
          GCHK(hipSetDevice(R.dev));
          GCHK(hipEventRecord(R.evSent[b], R.cs));
        }
    } else if (g->hostX) {
      // host transport (rank mode, one rank in this process): blocking, staged through pinned memory
      GRank& R = g->r[0];
      GCHK(hipSetDevice(R.dev));
      const size_t ab = sizeof(int32_t), cb = 3 * sizeof(float);
      if (R.rank != 0) {
        const size_t n = R.hAll.size();
        if (n) {
          GCHK(hipMemcpyAsync(g->hSend, R.sArgb[b], n * ab, hipMemcpyDeviceToHost, R.cs));
          if (g->rgb) GCHK(hipMemcpyAsync(g->hSend + n * ab, R.sRgb[b], n * cb, hipMemcpyDeviceToHost, R.cs));
        }
        GCHK(hipEventRecord(R.evSent[b], R.cs));
        GCHK(hipStreamSynchronize(R.cs));
        if (n && ((rc = comm_send(g->comm, g->hSend, n * ab, 0)) ||
                  (g->rgb && (rc = comm_send(g->comm, g->hSend + n * ab, n * cb, 0)))))
          return rc;
      } else {
        // the previous frame's upload from hRecv has finished once cs is idle; slab b's last scatter
        // is ordered before this frame's upload by evRecv[b]
        GCHK(hipStreamSynchronize(R.cs));
        for (int q = 1; q < g->world; ++q) {
          const int64_t o = recv_offset(g, q);
          const size_t n = (size_t)g->npix[q];
          if (!n) continue;
          if ((rc = comm_recv(g->comm, g->hRecv + o * ab, n * ab, q))) return rc;
          if (g->rgb && (rc = comm_recv(g->comm, g->hRecv + g->nRecv * ab + o * cb, n * cb, q))) return rc;
        }
        GCHK(hipStreamWaitEvent(R.cs, g->evRecv[b], 0));
        if (g->nRecv) {
          GCHK(hipMemcpyAsync(g->rArgb[b], g->hRecv, g->nRecv * ab, hipMemcpyHostToDevice, R.cs));
          if (g->rgb) GCHK(hipMemcpyAsync(g->rRgb[b], g->hRecv + g->nRecv * ab, g->nRecv * cb, hipMemcpyHostToDevice, R.cs));
        }
      }
    } else {
      // one process: device copies of every rank's packed pixels into rank 0's receive slab
      GCHK(hipSetDevice(R0->dev));
      for (GRank& R : g->r) {
        const size_t n = R.hAll.size();
        if (R.rank == 0) continue;
        GCHK(hipSetDevice(R.dev));
        GCHK(hipStreamWaitEvent(R.cs, g->evRecv[b], 0));
        if (n) {
          GCHK(hipMemcpyPeerAsync(g->rArgb[b] + R.off, g->rootDev, R.sArgb[b], R.dev, n * sizeof(int32_t), R.cs));
          if (g->rgb)
            GCHK(hipMemcpyPeerAsync(g->rRgb[b] + 3 * R.off, g->rootDev, R.sRgb[b], R.dev, n * 3 * sizeof(float), R.cs));
        }
        GCHK(hipEventRecord(R.evSent[b], R.cs));
        GCHK(hipEventRecord(g->evCopied[R.rank], R.cs));
      }
      GCHK(hipSetDevice(R0->dev));
      for (GRank& R : g->r)
        if (R.rank != 0) GCHK(hipStreamWaitEvent(R0->cs, g->evCopied[R.rank], 0));
    }
    if (R0) {
      GCHK(hipSetDevice(R0->dev));
      if ((rc = enqueue_scatter(g, R0->cs, b, 0, g->nRecv, rgb, argb))) return rc;
      GCHK(hipEventRecord(g->evRecv[b], R0->cs));
    }
  }
  if (R0) {  // the frame is complete when rank 0's own render and the scatter are
    GCHK(hipSetDevice(R0->dev));
    GCHK(hipEventRecord(R0->evRendered, R0->st));
    GCHK(hipStreamWaitEvent(R0->cs, R0->evRendered, 0));
  }
  g->frame++;
  return RT_OK;
}

int sync_group(rt_group* g) {
  for (GRank& R : g->r) {
    GCHK(hipSetDevice(R.dev));
    GCHK(hipStreamSynchronize(R.side));
    GCHK(hipStreamSynchronize(R.st));
    GCHK(hipStreamSynchronize(R.cs));
  }
  return RT_OK;
}

int destroy_group(rt_group* g) {
  if (!g) return RT_OK;
  for (GRank& R : g->r) {
    (void)hipSetDevice(R.dev);
    if (R.side) (void)hipStreamSynchronize(R.side);
    if (R.st) (void)hipStreamSynchronize(R.st);
    if (R.cs) (void)hipStreamSynchronize(R.cs);
  }
  for (GRank& R : g->r) {
    (void)hipSetDevice(R.dev);
    if (R.nccl && !g->rankMode && g_rccl.ok) (void)g_rccl.commDestroy(R.nccl);  // rank mode: the rt_comm's
    for (hipEvent_t e : {R.evStart, R.evSide, R.evRendered, R.evSent[0], R.evSent[1], R.evFree[0], R.evFree[1]})
      if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < KRING; ++k) {
      if (R.tA[k]) (void)hipEventDestroy(R.tA[k]);
      if (R.tB[k]) (void)hipEventDestroy(R.tB[k]);
    }
    if (R.st) (void)hipStreamDestroy(R.st);
    if (R.side) (void)hipStreamDestroy(R.side);
    if (R.cs) (void)hipStreamDestroy(R.cs);
  }
  for (hipEvent_t e : g->evCopied)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : g->evRecv)
    if (e) (void)hipEventDestroy(e);
  for (void* p : g->allocs) (void)hipFree(p);
  for (void* p : g->planAllocs) (void)hipFree(p);
  for (void* p : g->planHost) (void)hipHostFree(p);
  if (g->stage) (void)hipHostFree(g->stage);
  if (g->ownComm) rt_comm_destroy(g->comm);
  delete g;
  return RT_OK;
}
}  // namespace

extern "C" {

int rt_rank_plan(const uint32_t* cost, const double* weight, int ntiles, int world, double heavy, int slots,
                 int32_t* owner, int32_t* order) {
  if (ntiles < 0 || world < 1 || (ntiles > 0 && (!cost || !owner || !order)))
    return set_error(RT_E_INVALID, "rt_rank_plan: bad arguments");
  if (!(heavy > 0)) heavy = 1.25;
  if (slots <= 0) slots = 4096;
  plan_ranks(cost, ntiles, world, heavy, slots, owner, order, weight);
  return RT_OK;
}

int rt_group_unique_id(void* id, int cap) {
  if (!id || cap < (int)sizeof(ncclUniqueId)) return set_error(RT_E_INVALID, "rt_group_unique_id: buffer < 128 bytes");
  int rc = rccl_load();
  if (rc) return rc;
  ncclUniqueId u;
  const ncclResult_t nr = g_rccl.getUniqueId(&u);
  if (nr != ncclSuccess) return set_error(RT_E_HIP, std::string("ncclGetUniqueId failed: ") + g_rccl.errStr(nr));
  std::memcpy(id, &u, sizeof(u));
  return (int)sizeof(u);
}

int rt_group_create(rt_scene* const* scenes, int n, const rt_render_params* p, uint32_t flags, double heavy, int slots,
                    rt_group** out) {
  if (!scenes || n < 1 || !out) return set_error(RT_E_INVALID, "rt_group_create: bad arguments");
  *out = nullptr;
  DeviceGuard dg;
  for (int i = 0; i < n; ++i)
    if (!scenes[i]) return set_error(RT_E_INVALID, "rt_group_create: null scene");
  const bool rccl = n > 1 && !(flags & RT_GROUP_COPY);
  if (rccl) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j)
        if (scenes[i]->device == scenes[j]->device)
          return set_error(RT_E_INVALID, "rt_group_create: the RCCL transport needs one device per rank (RT_GROUP_COPY shares)");
    int rc = rccl_load();
    if (rc) return rc;
  }
  rt_group* g = new rt_group();
  g->world = n;
  g->useRccl = rccl;
  g->root = true;
  g->rootDev = scenes[0]->device;
  int rc = make_layout(g, scenes[0], p, flags);
  std::vector<uint32_t> cost;
  if (rc == RT_OK) {
    cost.assign(g->ntiles, 1);
    const int m = rt_tile_costs(scenes[0], &g->p, cost.data(), g->ntiles);
    rc = m < 0 ? m : (m != g->ntiles ? set_error(RT_E_INVALID, "rt_group_create: tile count mismatch") : RT_OK);
  }
  if (rc == RT_OK) rc = make_plan(g, cost, heavy, slots);
  if (rc == RT_OK) {
    g->r.resize(n);
    for (int i = 0; i < n; ++i) {
      g->r[i].s = scenes[i];
      g->r[i].dev = scenes[i]->device;
      g->r[i].rank = i;
    }
    rc = setup_ranks(g);
  }
  if (rc == RT_OK && rccl) {
    std::vector<ncclComm_t> comms(n);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = g->r[i].dev;
    ncclResult_t nr = g_rccl.commInitAll(comms.data(), n, devs.data());
    if (nr != ncclSuccess) rc = set_error(RT_E_HIP, std::string("ncclCommInitAll failed: ") + g_rccl.errStr(nr));
    else
      for (int i = 0; i < n; ++i) g->r[i].nccl = comms[i];
  }
  if (rc != RT_OK) {
    const std::string msg = rt_last_error();
    destroy_group(g);
    return set_error(rc, msg);
  }
  *out = g;
  return RT_OK;
}

int rt_group_create_comm(rt_scene* scene, rt_comm* comm, const rt_render_params* p, uint32_t flags, double heavy,
                         int slots, rt_group** out) {
  if (!scene || !out) return set_error(RT_E_INVALID, "rt_group_create_comm: bad arguments");
  *out = nullptr;
  DeviceGuard dg;
  const int world = comm ? comm->world : 1, rank = comm ? comm->rank : 0;
  if (flags & RT_GROUP_COPY) return set_error(RT_E_INVALID, "rt_group_create_comm: RT_GROUP_COPY is a one-process transport");
  rt_group* g = new rt_group();
  g->world = world;
  g->rankMode = true;
  g->comm = world > 1 ? comm : nullptr;
  g->useRccl = world > 1 && comm->rccl;
  g->hostX = world > 1 && !comm->rccl;
  g->root = rank == 0;
  g->rootDev = scene->device;
  int rc = (g->useRccl && comm->device != scene->device)
               ? set_error(RT_E_INVALID, "rt_group_create_comm: the RCCL communicator is on device " +
                                             std::to_string(comm->device) + ", the scene on " + std::to_string(scene->device))
               : RT_OK;
  if (rc == RT_OK) rc = make_layout(g, scene, p, flags);
  if (rc == RT_OK && !(heavy > 0)) heavy = 1.25;
  if (rc == RT_OK && slots <= 0) slots = 4096;
  // 1. the ranks were given the same frame (a mismatch would size the collectives differently)
  if (g->comm) {
    int64_t hb;
    std::memcpy(&hb, &heavy, sizeof(hb));
    const int64_t mine[10] = {rc, g->W, g->H, g->p.spp, (int64_t)g->p.seed, g->p.flags, hb, slots, g->ntiles, g->rgb};
    const std::string myMsg = rc ? std::string(rt_last_error()) : std::string();
    std::vector<int64_t> all(10 * (size_t)world);
    int rc2 = comm_allgather(g->comm, mine, all.data(), sizeof(mine));
    if (rc2 == RT_OK && rc) rc2 = set_error(rc, myMsg);
    for (int q = 0; q < world && rc2 == RT_OK; ++q) {
      const int64_t* x = &all[10 * (size_t)q];
      if (x[0]) rc2 = set_error((int)x[0], "rt_group_create_comm: rank " + std::to_string(q) + " failed its setup");
      else if (std::memcmp(x + 1, mine + 1, 9 * sizeof(int64_t)))
        rc2 = set_error(RT_E_INVALID, "rt_group_create_comm: rank " + std::to_string(q) +
                                          " was given a different frame (size / spp / seed / flags / heavy / slots)");
    }
    rc = rc2;
  }
  // 2. rank 0 measures the layout's wave times; every rank receives them behind rank 0's status
  std::vector<uint32_t> cost;
  if (rc == RT_OK) {
    cost.assign(g->ntiles + 1, 1);
    cost[0] = 0;
    if (rank == 0) {
      const int m = rt_tile_costs(scene, &g->p, cost.data() + 1, g->ntiles);
      const int crc = m < 0 ? m : (m != g->ntiles ? set_error(RT_E_INVALID, "rt_group_create_comm: tile count mismatch") : RT_OK);
      cost[0] = (uint32_t)crc;
      if (crc) std::fill(cost.begin() + 1, cost.end(), 1u);
    }
    const std::string msg0 = cost[0] ? std::string(rt_last_error()) : std::string();
    if (g->comm) rc = comm_bcast(g->comm, cost.data(), cost.size() * sizeof(uint32_t), 0);
    if (rc == RT_OK && cost[0])
      rc = rank == 0 ? set_error((int)(int32_t)cost[0], msg0)
                     : set_error((int)(int32_t)cost[0], "rt_group_create_comm: rank 0 failed to calibrate the layout");
    cost.erase(cost.begin());
  }
  // 3. the plan (deterministic: every rank derives the same one) and this rank's lists, checked
  if (rc == RT_OK) rc = make_plan(g, cost, heavy, slots);
  if (rc == RT_OK) {
    GRank R;
    R.s = scene;
    R.dev = scene->device;
    R.rank = rank;
    R.nccl = g->useRccl ? comm->nccl : nullptr;
    g->r.push_back(R);
    rc = setup_ranks(g);  // collective (plan_check)
  }
  if (rc != RT_OK) {
    const std::string msg = rt_last_error();
    destroy_group(g);
    return set_error(rc, msg);
  }
  *out = g;
  return RT_OK;
}

int rt_group_create_rank(rt_scene* scene, int rank, int world, const void* unique_id, const rt_render_params* p,
                         uint32_t flags, double heavy, int slots, rt_group** out) {
  if (!scene || !out || world < 1 || rank < 0 || rank >= world || (world > 1 && !unique_id))
    return set_error(RT_E_INVALID, "rt_group_create_rank: bad arguments");
  *out = nullptr;
  rt_comm* c = nullptr;
  if (world > 1) {
    int rc = rt_comm_create_rccl(rank, world, unique_id, scene->device, &c);
    if (rc) return rc;
  }
  int rc = rt_group_create_comm(scene, c, p, flags, heavy, slots, out);
  if (rc) {
    const std::string msg = rt_last_error();
    rt_comm_destroy(c);
    return set_error(rc, msg);
  }
  (*out)->ownComm = c != nullptr;
  return RT_OK;
}

int rt_group_render(rt_group* g, float* d_rgb, int32_t* d_argb) {
  if (!g) return set_error(RT_E_INVALID, "rt_group_render: null group");
  DeviceGuard dg;
  return group_frame(g, d_rgb, d_argb);
}

int rt_group_sync(rt_group* g) {
  if (!g) return set_error(RT_E_INVALID, "rt_group_sync: null group");
  DeviceGuard dg;
  return sync_group(g);
}

int rt_group_render_host(rt_group* g, float* rgb, int32_t* argb) {
  if (!g) return set_error(RT_E_INVALID, "rt_group_render_host: null group");
  DeviceGuard dg;
  if (rgb && !g->rgb) return set_error(RT_E_INVALID, "rt_group_render_host: float-RGB output needs RT_GROUP_RGB");
  int rc = group_frame(g, g->root ? g->outRgb : nullptr, g->root ? g->outArgb : nullptr);
  if (rc) return rc;
  if (!g->root) return sync_group(g);
  GRank* R0 = local_rank(g, 0);
  const size_t npx = (size_t)g->W * g->H;
  const size_t na = argb ? npx * sizeof(int32_t) : 0, nr = rgb ? npx * 3 * sizeof(float) : 0;
  GCHK(hipSetDevice(R0->dev));
  if (!g->stage && (na + nr) > 0) GCHK(hipHostMalloc(&g->stage, npx * (sizeof(int32_t) + (g->rgb ? 3 * sizeof(float) : 0))));
  char* stg = (char*)g->stage;
  if (argb) GCHK(hipMemcpyAsync(stg, g->outArgb, na, hipMemcpyDeviceToHost, R0->cs));
  if (rgb) GCHK(hipMemcpyAsync(stg + na, g->outRgb, nr, hipMemcpyDeviceToHost, R0->cs));
  if ((rc = sync_group(g))) return rc;
  if (argb) std::memcpy(argb, stg, na);
  if (rgb) std::memcpy(rgb, stg + na, nr);
  return RT_OK;
}

int rt_group_frame(rt_group* g, float** d_rgb, int32_t** d_argb) {
  if (!g) return set_error(RT_E_INVALID, "rt_group_frame: null group");
  if (d_rgb) *d_rgb = g->root ? g->outRgb : nullptr;
  if (d_argb) *d_argb = g->root ? g->outArgb : nullptr;
  return RT_OK;
}

int rt_group_info(const rt_group* g, int64_t* info, int n) {
  if (!g || !info) return set_error(RT_E_INVALID, "rt_group_info: null argument");
  const int64_t v[10] = {g->world, (int64_t)g->r.size(), g->r.empty() ? -1 : g->r[0].rank, g->ntiles, g->tilesX, g->tw,
                         g->th, g->useRccl ? 1 : (g->hostX ? 2 : 0), g->frame, g->planChecks};
  for (int i = 0; i < n && i < 10; ++i) info[i] = v[i];
  return RT_OK;
}

int rt_group_plan(const rt_group* g, int32_t* owner, int32_t* order, int cap) {
  if (!g) return set_error(RT_E_INVALID, "rt_group_plan: null group");
  for (int i = 0; i < g->ntiles && i < cap; ++i) {
    if (owner) owner[i] = g->owner[i];
    if (order) order[i] = g->order[i];
  }
  return g->ntiles;
}

int rt_group_rank_pixels(const rt_group* g, int rank, int32_t* pixels, int64_t cap) {
  if (!g || rank < 0 || rank >= g->world) return set_error(RT_E_INVALID, "rt_group_rank_pixels: bad arguments");
  std::vector<int32_t> a, b, c, d;
  rank_lists(g, rank, a, b, c, d);
  for (int64_t i = 0; i < (int64_t)d.size() && i < cap && pixels; ++i) pixels[i] = d[i];
  return (int)std::min<int64_t>(d.size(), INT32_MAX);
}

int rt_group_kernel_ms(rt_group* g, int rank, double* avg_ms, int* frames) {
  if (!g || !avg_ms) return set_error(RT_E_INVALID, "rt_group_kernel_ms: null argument");
  DeviceGuard dg;
  GRank* R = local_rank(g, rank);
  if (!R) return set_error(RT_E_INVALID, "rt_group_kernel_ms: rank not driven by this process");
  GCHK(hipSetDevice(R->dev));
  GCHK(hipStreamSynchronize(R->st));
  const int64_t m = std::min<int64_t>(R->timed, KRING);
  double sum = 0;
  for (int64_t k = 0; k < m; ++k) {
    const int64_t f = R->timed - 1 - k;
    float ms = 0;
    GCHK(hipEventElapsedTime(&ms, R->tA[f % KRING], R->tB[f % KRING]));
    sum += ms;
  }
  *avg_ms = m ? sum / m : 0.0;
  if (frames) *frames = (int)m;
  R->timed = 0;
  return RT_OK;
}

// One rank's step alone (the one-process emulation on one GPU): its render, pack,
// copy into rank 0's slab and the scatter of its slice -- rank 0: its render and the scatter of the
// whole slab -- frames pipelined as rt_group_render pipelines them; wall-clock time per step and the
// mean HIP-event time of its render.
int rt_group_time_rank(rt_group* g, int rank, int warmup, int iters, double* step_ms, double* kernel_ms) {
  if (!g || iters <= 0 || !step_ms || !kernel_ms) return set_error(RT_E_INVALID, "rt_group_time_rank: bad arguments");
  DeviceGuard dg;
  if (g->rankMode || g->useRccl) return set_error(RT_E_INVALID, "rt_group_time_rank: one-process RT_GROUP_COPY groups only");
  GRank* R = local_rank(g, rank);
  GRank* R0 = local_rank(g, 0);
  if (!R || !R0) return set_error(RT_E_INVALID, "rt_group_time_rank: bad rank");
  int rc;
  auto step = [&](int64_t f) -> int {
    const int b = (int)(f & 1);
    if (rank == 0) {
      if ((rc = enqueue_render(g, *R, g->outRgb, g->outArgb, true))) return rc;
      GCHK(hipSetDevice(R0->dev));
      GCHK(hipStreamWaitEvent(R0->cs, g->evRecv[b], 0));
      if ((rc = enqueue_scatter(g, R0->cs, b, 0, g->nRecv, g->outRgb, g->outArgb))) return rc;
      GCHK(hipEventRecord(g->evRecv[b], R0->cs));
      return RT_OK;
    }
    if ((rc = enqueue_rank_render(g, *R, b, true)) || (rc = enqueue_pack(g, *R, b))) return rc;
    const size_t n = R->hAll.size();
    GCHK(hipStreamWaitEvent(R->cs, g->evRecv[b], 0));
    if (n) {
      GCHK(hipMemcpyPeerAsync(g->rArgb[b] + R->off, g->rootDev, R->sArgb[b], R->dev, n * sizeof(int32_t), R->cs));
      if (g->rgb) GCHK(hipMemcpyPeerAsync(g->rRgb[b] + 3 * R->off, g->rootDev, R->sRgb[b], R->dev, n * 12, R->cs));
    }
    GCHK(hipEventRecord(R->evSent[b], R->cs));
    if (R->dev == R0->dev) {
      if ((rc = enqueue_scatter(g, R->cs, b, R->off, R->off + (int64_t)n, g->outRgb, g->outArgb))) return rc;
      GCHK(hipEventRecord(g->evRecv[b], R->cs));
    }
    return RT_OK;
  };
  for (int i = 0; i < warmup; ++i)
    if ((rc = step(i))) return rc;
  if ((rc = sync_group(g))) return rc;
  R->timed = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i)
    if ((rc = step(warmup + i))) return rc;
  if ((rc = sync_group(g))) return rc;
  const auto t1 = std::chrono::steady_clock::now();
  *step_ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / iters;
  int fr = 0;
  return rt_group_kernel_ms(g, rank, kernel_ms, &fr);
}

int rt_group_count(rt_group* g, int rank, uint64_t* stats) {
  if (!g || !stats) return set_error(RT_E_INVALID, "rt_group_count: null argument");
  GRank* R = local_rank(g, rank);
  if (!R) return set_error(RT_E_INVALID, "rt_group_count: rank not driven by this process");
  std::vector<int32_t> t = R->hTiles;
  t.insert(t.end(), R->hSplit.begin(), R->hSplit.end());
  for (int i = 0; i < RT_ST_N; ++i) stats[i] = 0;
  if (t.empty()) return RT_OK;
  return rt_render_tiles_count(R->s, &g->p, t.data(), (int)t.size(), stats);
}

// Re-cut the plan from the ranks' measured render times (collective in rank mode). The cost model
// (a tile's measured wave time in the 1-GPU calibration) predicts a rank's kernel imperfectly -- waves
// running together share caches and CUs differently in a rank's compact region than in the whole
// frame -- so each round times every rank's render (iters frames, HIP events; in the one-process
// emulation one rank at a time, each with the whole GPU), folds the rank's time per unit of
// predicted cost into its tiles' cut weights, and cuts again. The split tiles and the dispatch order
// stay those of the measured wave times; only the cut moves. rank_ms[0..world) (may be NULL) gets the
// render times of the last measurement, taken after the last cut.
int rt_group_rebalance(rt_group* g, int rounds, int iters, double* rank_ms) {
  if (!g || rounds < 0 || iters <= 0) return set_error(RT_E_INVALID, "rt_group_rebalance: bad arguments");
  DeviceGuard dg;
  if (g->weight.empty()) g->weight.assign(g->ntiles, 1.0);
  std::vector<double> T(g->world, 0.0);
  const bool coll = g->rankMode && g->world > 1 && g->comm;
  for (int round = 0; round <= rounds; ++round) {
    // this process's ranks, each alone (one-process groups share devices), after 3 untimed frames;
    // in rank mode a local failure is carried into the all-gather below instead of returning early
    auto time_ranks = [&]() -> int {
      int rc = sync_group(g);
      if (rc) return rc;
      for (GRank& R : g->r) {
        const bool r0 = R.rank == 0;
        for (int i = 0; i < 3; ++i)
          if ((rc = enqueue_render(g, R, r0 ? g->outRgb : R.fRgb[0], r0 ? g->outArgb : R.fArgb[0], false))) return rc;
        GCHK(hipSetDevice(R.dev));
        GCHK(hipStreamSynchronize(R.st));
        R.timed = 0;
        for (int i = 0; i < iters; ++i)
          if ((rc = enqueue_render(g, R, r0 ? g->outRgb : R.fRgb[0], r0 ? g->outArgb : R.fArgb[0], true))) return rc;
        int fr = 0;
        if ((rc = rt_group_kernel_ms(g, R.rank, &T[R.rank], &fr))) return rc;
      }
      return RT_OK;
    };
    int rc = time_ranks();
    if (coll) {  // every rank's {status, time} to every rank
      const std::string mine = rc ? std::string(rt_last_error()) : std::string();
      const GRank& R = g->r[0];
      double rec[2] = {(double)rc, T[R.rank]};
      std::vector<double> all(2 * (size_t)g->world);
      int rc2 = comm_allgather(g->comm, rec, all.data(), sizeof(rec));
      if (rc2) return rc2;
      if (rc) return set_error(rc, mine);
      for (int q = 0; q < g->world; ++q) {
        if (all[2 * q] != 0)
          return set_error((int)all[2 * q], "rt_group_rebalance: rank " + std::to_string(q) + " failed to time its render");
        T[q] = all[2 * q + 1];
      }
    } else if (rc) {
      return rc;
    }
    if (round == rounds) break;
    // a rank's time per unit of weighted cost, relative to the frame's
    std::vector<double> C(g->world, 0.0);
    for (int t = 0; t < g->ntiles; ++t) C[g->owner[t] % g->world] += (double)g->cost[t] * g->weight[t];
    double Tsum = 0, Csum = 0;
    for (int q = 0; q < g->world; ++q) { Tsum += T[q]; Csum += C[q]; }
    if (!(Tsum > 0) || !(Csum > 0)) break;
    std::vector<double> f(g->world, 1.0);  // damped (^0.75): the measured times carry a few % of noise
    for (int q = 0; q < g->world; ++q)
      if (C[q] > 0 && T[q] > 0) f[q] = std::pow((T[q] / Tsum) / (C[q] / Csum), 0.75);
    for (int t = 0; t < g->ntiles; ++t) g->weight[t] *= f[g->owner[t] % g->world];
    if ((rc = make_plan(g, g->cost, g->heavy, g->slots)) || (rc = setup_lists(g))) return rc;  // setup_lists: collective check
  }
  if (rank_ms)
    for (int q = 0; q < g->world; ++q) rank_ms[q] = T[q];
  return RT_OK;
}

void rt_group_destroy(rt_group* g) {
  DeviceGuard dg;
  (void)destroy_group(g);
}

int rt_group_rccl_selftest(int device, int n) {
  if (n < 1) return set_error(RT_E_INVALID, "rt_group_rccl_selftest: n < 1");
  DeviceGuard dg;
  int rc = rccl_load();
  if (rc) return rc;
  GCHK(hipSetDevice(device));
  std::vector<int32_t> h(n), back(4 * (size_t)n, 0);
  for (int i = 0; i < n; ++i) h[i] = (int32_t)(0x9E3779B9u * (uint32_t)(i + 1));
  int32_t* d = nullptr;  // [0, n) source, [n, 2n) broadcast, [2n, 3n) all-gather, [3n, 4n) received
  hipStream_t st = nullptr;
  ncclComm_t c1 = nullptr, c2 = nullptr;
  std::string err;
  auto hfail = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && err.empty()) err = std::string(what) + ": " + hipGetErrorString(e);
    return e != hipSuccess;
  };
  auto nfail = [&](ncclResult_t r, const char* what) {
    if (r != ncclSuccess && err.empty()) err = std::string(what) + ": " + g_rccl.errStr(r);
    return r != ncclSuccess;
  };
  do {
    if (hfail(hipMalloc(&d, 4 * sizeof(int32_t) * n), "hipMalloc")) break;
    if (hfail(hipMemset(d + n, 0, 3 * sizeof(int32_t) * n), "hipMemset")) break;
    if (hfail(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate")) break;
    if (hfail(hipMemcpy(d, h.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice), "hipMemcpy")) break;
    ncclUniqueId u;
    if (nfail(g_rccl.getUniqueId(&u), "ncclGetUniqueId")) break;
    if (nfail(g_rccl.commInitRank(&c1, 1, u, 0), "ncclCommInitRank")) break;
    int dev = device;
    if (nfail(g_rccl.commInitAll(&c2, 1, &dev), "ncclCommInitAll")) break;
    if (nfail(g_rccl.bcast(d, d + n, (size_t)n, ncclInt32, 0, c1, st), "ncclBroadcast")) break;
    if (nfail(g_rccl.allGather(d, d + 2 * n, (size_t)n, ncclInt32, c2, st), "ncclAllGather")) break;
    if (nfail(g_rccl.groupStart(), "ncclGroupStart")) break;
    ncclResult_t r1 = g_rccl.send(d, (size_t)n, ncclInt32, 0, c1, st);
    ncclResult_t r2 = g_rccl.recv(d + 3 * n, (size_t)n, ncclInt32, 0, c1, st);
    ncclResult_t r3 = g_rccl.groupEnd();
    if (nfail(r1, "ncclSend") || nfail(r2, "ncclRecv") || nfail(r3, "ncclGroupEnd")) break;
    if (hfail(hipStreamSynchronize(st), "hipStreamSynchronize")) break;
    if (hfail(hipMemcpy(back.data(), d, 4 * sizeof(int32_t) * n, hipMemcpyDeviceToHost), "hipMemcpy")) break;
    for (int k = 1; k < 4 && err.empty(); ++k)
      for (int i = 0; i < n; ++i)
        if (back[(size_t)k * n + i] != h[i]) {
          static const char* what[4] = {"", "ncclBroadcast", "ncclAllGather", "ncclSend / ncclRecv"};
          err = std::string(what[k]) + ": element " + std::to_string(i) + " differs";
          break;
        }
  } while (false);
  if (c1) (void)g_rccl.commDestroy(c1);
  if (c2) (void)g_rccl.commDestroy(c2);
  if (st) (void)hipStreamDestroy(st);
  if (d) (void)hipFree(d);
  return err.empty() ? RT_OK : set_error(RT_E_HIP, "rt_group_rccl_selftest: " + err);
}

}  // extern "C"
