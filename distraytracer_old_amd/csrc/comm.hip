// Communicators (rt_comm_*) and the sharded photon pre-pass (rt_photons_build_comm / _local).
//
// A communicator is the transport of a one-process-per-GPU group (group.hip) and of the photon
// pre-pass split over ranks. RCCL (ncclCommInitRank over the unique id rank 0 made)
// is the production transport: one device per rank, the frame exchange stream-ordered over xGMI. The
// host transport hands every collective to four caller callbacks on host buffers -- the JNI side's
// own sockets / MPI, or torch.distributed's gloo in the tests -- and lets ranks share a device, so
// the rank-mode code path (every collective, every offset) runs as N processes on one GPU.
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <set>
#include <vector>

#include "comm.h"

using namespace rt;

namespace rt {
RcclApi g_rccl;
static std::mutex g_rccl_mu;

int rccl_load() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  RcclApi& R = g_rccl;
  if (!R.tried) {
    R.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      R.why = std::string("cannot load librccl.so.1: ") + dlerror();
    } else {
      bool all = true;
      auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        all = all && fn != nullptr;
      };
      sym(R.getUniqueId, "ncclGetUniqueId");
      sym(R.commInitRank, "ncclCommInitRank");
      sym(R.commInitAll, "ncclCommInitAll");
      sym(R.commDestroy, "ncclCommDestroy");
      sym(R.groupStart, "ncclGroupStart");
      sym(R.groupEnd, "ncclGroupEnd");
      sym(R.send, "ncclSend");
      sym(R.recv, "ncclRecv");
      sym(R.bcast, "ncclBroadcast");
      sym(R.allGather, "ncclAllGather");
      sym(R.errStr, "ncclGetErrorString");
      R.ok = all;
      if (!all) R.why = "librccl.so.1 lacks an entry point the group needs";
    }
  }
  return R.ok ? RT_OK : set_error(RT_E_INVALID, "RCCL transport unavailable: " + R.why);
}

namespace {
int host_err(const char* what) { return set_error(RT_E_HIP, std::string(what) + ": the host transport's callback failed"); }

// RCCL: the staging buffer (grow-only) on the communicator's device
int stage(rt_comm* c, size_t bytes) {
  if (bytes <= c->dcap) return RT_OK;
  if (c->dbuf) (void)hipFree(c->dbuf);
  c->dbuf = nullptr;
  c->dcap = 0;
  hipError_t e = hipMalloc(&c->dbuf, bytes);
  if (e != hipSuccess) return set_error(RT_E_HIP, std::string("rt_comm staging: ") + hipGetErrorString(e));
  c->dcap = bytes;
  return RT_OK;
}

int rccl_fail(const char* what, hipError_t he, ncclResult_t nr) {
  if (he != hipSuccess) return set_error(RT_E_HIP, std::string(what) + ": " + hipGetErrorString(he));
  return set_error(RT_E_HIP, std::string(what) + ": " + g_rccl.errStr(nr));
}
}  // namespace

int comm_bcast(rt_comm* c, void* buf, size_t bytes, int root) {
  if (!c || c->world == 1 || bytes == 0) return RT_OK;
  if (!c->rccl) return c->ops.bcast(c->ops.ctx, buf, (int64_t)bytes, root) ? host_err("broadcast") : RT_OK;
  DeviceGuard dg;
  hipError_t he = hipSetDevice(c->device);
  int rc = he == hipSuccess ? stage(c, bytes) : RT_OK;
  if (rc) return rc;
  ncclResult_t nr = ncclSuccess;
  if (he == hipSuccess) he = hipMemcpy(c->dbuf, buf, bytes, hipMemcpyHostToDevice);
  if (he == hipSuccess) nr = g_rccl.bcast(c->dbuf, c->dbuf, bytes, ncclInt8, root, c->nccl, c->st);
  if (he == hipSuccess && nr == ncclSuccess) he = hipStreamSynchronize(c->st);
  if (he == hipSuccess && nr == ncclSuccess) he = hipMemcpy(buf, c->dbuf, bytes, hipMemcpyDeviceToHost);
  return (he != hipSuccess || nr != ncclSuccess) ? rccl_fail("rt_comm broadcast", he, nr) : RT_OK;
}

int comm_allgather(rt_comm* c, const void* in, void* out, size_t bytes) {
  if (!c || c->world == 1) {
    if (bytes) std::memmove(out, in, bytes);
    return RT_OK;
  }
  if (bytes == 0) return RT_OK;
  if (!c->rccl) return c->ops.allgather(c->ops.ctx, in, out, (int64_t)bytes) ? host_err("all-gather") : RT_OK;
  DeviceGuard dg;
  const size_t total = bytes * (size_t)c->world;
  hipError_t he = hipSetDevice(c->device);
  int rc = he == hipSuccess ? stage(c, total + bytes) : RT_OK;
  if (rc) return rc;
  char* d = (char*)c->dbuf;
  ncclResult_t nr = ncclSuccess;
  if (he == hipSuccess) he = hipMemcpy(d + total, in, bytes, hipMemcpyHostToDevice);
  if (he == hipSuccess) nr = g_rccl.allGather(d + total, d, bytes, ncclInt8, c->nccl, c->st);
  if (he == hipSuccess && nr == ncclSuccess) he = hipStreamSynchronize(c->st);
  if (he == hipSuccess && nr == ncclSuccess) he = hipMemcpy(out, d, total, hipMemcpyDeviceToHost);
  return (he != hipSuccess || nr != ncclSuccess) ? rccl_fail("rt_comm all-gather", he, nr) : RT_OK;
}

int comm_send(rt_comm* c, const void* buf, size_t bytes, int peer) {
  if (!c || c->rccl) return set_error(RT_E_INVALID, "comm_send: host transport only");
  if (bytes == 0) return RT_OK;
  return c->ops.send(c->ops.ctx, buf, (int64_t)bytes, peer) ? host_err("send") : RT_OK;
}

int comm_recv(rt_comm* c, void* buf, size_t bytes, int peer) {
  if (!c || c->rccl) return set_error(RT_E_INVALID, "comm_recv: host transport only");
  if (bytes == 0) return RT_OK;
  return c->ops.recv(c->ops.ctx, buf, (int64_t)bytes, peer) ? host_err("recv") : RT_OK;
}

int comm_all_ok(rt_comm* c, int local_rc, const char* what) {
  if (!c || c->world == 1) return local_rc;
  const std::string mine = local_rc ? std::string(rt_last_error()) : std::string();
  std::vector<int32_t> all(c->world, 0);
  const int32_t v = local_rc;
  int rc = comm_allgather(c, &v, all.data(), sizeof(int32_t));
  if (rc) return rc;
  if (local_rc) return set_error(local_rc, mine);
  for (int q = 0; q < c->world; ++q)
    if (all[q])
      return set_error(all[q], std::string(what) + ": rank " + std::to_string(q) + " failed (" + std::to_string(all[q]) +
                                   "); every rank stops here");
  return RT_OK;
}
}  // namespace rt

// ---------------------------------------------------------------------------------------------
// sharded photon pre-pass
namespace {
// the photon_list of n shards (rank order; each light-major, photon index ascending inside a light)
// in the reference's insertion order: light-major, then the shards' consecutive index ranges
void merge_shards(const std::vector<std::vector<double>>& pos, const std::vector<std::vector<double>>& pwr,
                  const std::vector<std::vector<int64_t>>& perLight, std::vector<double>& outPos,
                  std::vector<double>& outPwr) {
  const size_t L = perLight.empty() ? 0 : perLight[0].size();
  size_t total = 0;
  for (const auto& p : pos) total += p.size();
  outPos.clear();
  outPwr.clear();
  outPos.reserve(total);
  outPwr.reserve(total);
  std::vector<size_t> at(pos.size(), 0);
  for (size_t l = 0; l < L; ++l)
    for (size_t q = 0; q < pos.size(); ++q) {
      const size_t n3 = 3 * (size_t)perLight[q][l];
      outPos.insert(outPos.end(), pos[q].begin() + at[q], pos[q].begin() + at[q] + n3);
      outPwr.insert(outPwr.end(), pwr[q].begin() + at[q], pwr[q].begin() + at[q] + n3);
      at[q] += n3;
    }
}

// emitted photons of rank q's shard: [q P / N, (q + 1) P / N) of every light (multigpu.photon_shard)
void shard_range(int64_t P, int q, int n, int64_t& first, int64_t& count) {
  first = (int64_t)q * P / n;
  count = (int64_t)(q + 1) * P / n - first;
}
}  // namespace

extern "C" {

int rt_comm_create_rccl(int rank, int world, const void* unique_id, int device, rt_comm** out) {
  if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !unique_id))
    return set_error(RT_E_INVALID, "rt_comm_create_rccl: bad arguments");
  *out = nullptr;
  int rc = rccl_load();
  if (rc) return rc;
  DeviceGuard dg;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) return set_error(RT_E_HIP, std::string("rt_comm_create_rccl: ") + hipGetErrorString(he));
  rt_comm* c = new rt_comm();
  c->rank = rank;
  c->world = world;
  c->rccl = true;
  c->device = device;
  he = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking);
  ncclResult_t nr = ncclSuccess;
  if (he == hipSuccess) {
    ncclUniqueId u;
    if (world > 1) {
      std::memcpy(&u, unique_id, sizeof(u));
    } else {
      nr = g_rccl.getUniqueId(&u);
    }
    if (nr == ncclSuccess) nr = g_rccl.commInitRank(&c->nccl, world, u, rank);
  }
  if (he != hipSuccess || nr != ncclSuccess) {
    rc = he != hipSuccess ? set_error(RT_E_HIP, std::string("rt_comm_create_rccl: ") + hipGetErrorString(he))
                          : set_error(RT_E_HIP, std::string("ncclCommInitRank failed: ") + g_rccl.errStr(nr));
    rt_comm_destroy(c);
    return rc;
  }
  *out = c;
  return RT_OK;
}

int rt_comm_create_host(int rank, int world, const rt_comm_ops* ops, rt_comm** out) {
  if (!out || !ops || world < 1 || rank < 0 || rank >= world || !ops->bcast || !ops->allgather || !ops->send ||
      !ops->recv)
    return set_error(RT_E_INVALID, "rt_comm_create_host: bad arguments (every callback is required)");
  rt_comm* c = new rt_comm();
  c->rank = rank;
  c->world = world;
  c->rccl = false;
  c->ops = *ops;
  *out = c;
  return RT_OK;
}

int rt_comm_info(const rt_comm* c, int64_t* info, int n) {
  if (!c || !info) return set_error(RT_E_INVALID, "rt_comm_info: null argument");
  const int64_t v[4] = {c->rank, c->world, c->rccl ? 1 : 2, c->rccl ? c->device : -1};
  for (int i = 0; i < n && i < 4; ++i) info[i] = v[i];
  return RT_OK;
}

void rt_comm_destroy(rt_comm* c) {
  if (!c) return;
  DeviceGuard dg;
  if (c->rccl) {
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->nccl && g_rccl.ok) (void)g_rccl.commDestroy(c->nccl);
    if (c->st) (void)hipStreamDestroy(c->st);
    if (c->dbuf) (void)hipFree(c->dbuf);
  }
  delete c;
}

int rt_comm_selftest(rt_comm* c, int n) {
  if (!c || n < 1) return set_error(RT_E_INVALID, "rt_comm_selftest: bad arguments");
  const int world = c->world, rank = c->rank;
  auto val = [](int q, int i) { return (int32_t)(0x9E3779B9u * (uint32_t)(q + 1) ^ (uint32_t)(i * 2654435761u)); };
  std::vector<int32_t> mine(n), all((size_t)n * world, 0), buf(n);
  for (int i = 0; i < n; ++i) mine[i] = val(rank, i);
  int rc = comm_allgather(c, mine.data(), all.data(), sizeof(int32_t) * n);
  if (rc) return rc;
  for (int q = 0; q < world; ++q)
    for (int i = 0; i < n; ++i)
      if (all[(size_t)q * n + i] != val(q, i))
        return set_error(RT_E_HIP, "rt_comm_selftest: all-gather: rank " + std::to_string(q) + " element " + std::to_string(i));
  for (int root = 0; root < world; ++root) {  // every rank broadcasts once
    for (int i = 0; i < n; ++i) buf[i] = rank == root ? val(root, i) : 0;
    if ((rc = comm_bcast(c, buf.data(), sizeof(int32_t) * n, root))) return rc;
    for (int i = 0; i < n; ++i)
      if (buf[i] != val(root, i))
        return set_error(RT_E_HIP, "rt_comm_selftest: broadcast from rank " + std::to_string(root) + " element " + std::to_string(i));
  }
  if (!c->rccl && world > 1) {  // the group's exchange pattern: ranks > 0 to rank 0 in rank order, and back
    if (rank == 0) {
      for (int q = 1; q < world; ++q) {
        if ((rc = comm_recv(c, buf.data(), sizeof(int32_t) * n, q))) return rc;
        for (int i = 0; i < n; ++i)
          if (buf[i] != val(q, i)) return set_error(RT_E_HIP, "rt_comm_selftest: recv from rank " + std::to_string(q));
      }
      for (int q = 1; q < world; ++q) {
        for (int i = 0; i < n; ++i) buf[i] = val(q, i) ^ 0x5A5A5A5A;
        if ((rc = comm_send(c, buf.data(), sizeof(int32_t) * n, q))) return rc;
      }
    } else {
      if ((rc = comm_send(c, mine.data(), sizeof(int32_t) * n, 0))) return rc;
      if ((rc = comm_recv(c, buf.data(), sizeof(int32_t) * n, 0))) return rc;
      for (int i = 0; i < n; ++i)
        if (buf[i] != (val(rank, i) ^ 0x5A5A5A5A)) return set_error(RT_E_HIP, "rt_comm_selftest: recv from rank 0");
    }
  }
  return comm_all_ok(c, RT_OK, "rt_comm_selftest");
}

int rt_photons_build_comm(rt_scene* s, rt_comm* c, uint64_t seed) {
  if (!s) return set_error(RT_E_INVALID, "rt_photons_build_comm: null scene");
  if (!c || c->world == 1) return rt_photons_build(s, seed);
  DeviceGuard dg;
  HostScene& h = s->hs;
  const int world = c->world, rank = c->rank;
  // 1. every rank's shard (a rank's local failure is reported inside the header all-gather)
  int rc = h.photonMode ? check_photon_params(h) : RT_OK;
  std::vector<double> pos, pwr;
  std::vector<int64_t> per;
  if (rc == RT_OK && h.photonMode) {
    int64_t first, count;
    shard_range(h.photonCount, rank, world, first, count);
    rc = shoot_photons(s, seed, first, count, pos, pwr, per);
  }
  // 2. headers {status, lights, records, photons emitted, photon mode}: the ranks must hold the same scene
  constexpr int HN = 5;
  const int64_t mine[HN] = {rc, (int64_t)h.light.size(), (int64_t)(pos.size() / 3), h.photonCount, h.photonMode};
  const std::string myMsg = rc ? std::string(rt_last_error()) : std::string();
  std::vector<int64_t> hdr(HN * (size_t)world);
  int rc2 = comm_allgather(c, mine, hdr.data(), sizeof(mine));
  if (rc2) return rc2;
  if (rc) return set_error(rc, myMsg);
  for (int q = 0; q < world; ++q) {
    if (hdr[HN * q])
      return set_error((int)hdr[HN * q], "rt_photons_build_comm: rank " + std::to_string(q) + " failed its shard");
    if (hdr[HN * q + 1] != mine[1] || hdr[HN * q + 3] != mine[3] || hdr[HN * q + 4] != mine[4])
      return set_error(RT_E_INVALID, "rt_photons_build_comm: rank " + std::to_string(q) +
                                         " holds a different scene (lights / photon count / mode differ)");
  }
  if (!h.photonMode) return RT_OK;  // no photon map on any rank (rt_photons_build's no-op)
  const size_t L = (size_t)mine[1];
  // 3. per-light counts, then every shard's records broadcast from its rank (exact sizes, no padding)
  std::vector<int64_t> perAll(L * world, 0);
  per.resize(L, 0);
  if (L && (rc = comm_allgather(c, per.data(), perAll.data(), sizeof(int64_t) * L))) return rc;
  std::vector<std::vector<double>> P(world), W(world);
  std::vector<std::vector<int64_t>> PL(world);
  for (int q = 0; q < world; ++q) {
    const size_t n3 = 3 * (size_t)hdr[HN * q + 2];
    PL[q].assign(perAll.begin() + q * L, perAll.begin() + (q + 1) * L);
    int64_t sum = 0;
    for (int64_t v : PL[q]) sum += v;
    if (sum != hdr[HN * q + 2]) return set_error(RT_E_INVALID, "rt_photons_build_comm: inconsistent shard counts");
    if (q == rank) {
      P[q].swap(pos);
      W[q].swap(pwr);
    } else {
      P[q].assign(n3, 0.0);
      W[q].assign(n3, 0.0);
    }
    if ((rc = comm_bcast(c, P[q].data(), n3 * sizeof(double), q)) || (rc = comm_bcast(c, W[q].data(), n3 * sizeof(double), q)))
      return rc;
  }
  // 4. the reference's photon_list, and the same map on every rank
  std::vector<double> fullPos, fullPwr;
  merge_shards(P, W, PL, fullPos, fullPwr);
  if (fullPos.size() / 3 > (size_t)(INT32_MAX / 4)) return set_error(RT_E_INVALID, "photon map too large");
  s->photonsUploaded = false;
  return set_photon_map(s, fullPos, fullPwr);
}

int rt_photons_build_local(rt_scene* const* scenes, int n, uint64_t seed) {
  if (!scenes || n < 1) return set_error(RT_E_INVALID, "rt_photons_build_local: bad arguments");
  for (int q = 0; q < n; ++q)
    if (!scenes[q]) return set_error(RT_E_INVALID, "rt_photons_build_local: null scene");
  DeviceGuard dg;
  const HostScene& h0 = scenes[0]->hs;
  int rc = h0.photonMode ? check_photon_params(h0) : set_error(RT_E_INVALID, "rt_photons_build_local: scene has no photon map");
  if (rc) return rc;
  for (int q = 1; q < n; ++q)
    if (scenes[q]->hs.light.size() != h0.light.size() || scenes[q]->hs.photonCount != h0.photonCount)
      return set_error(RT_E_INVALID, "rt_photons_build_local: the scenes differ (lights / photon count)");
  std::vector<std::vector<double>> P(n), W(n);
  std::vector<std::vector<int64_t>> PL(n);
  for (int q = 0; q < n; ++q) {
    int64_t first, count;
    shard_range(h0.photonCount, q, n, first, count);
    if ((rc = shoot_photons(scenes[q], seed, first, count, P[q], W[q], PL[q]))) return rc;
  }
  std::vector<double> fullPos, fullPwr;
  merge_shards(P, W, PL, fullPos, fullPwr);
  if (fullPos.size() / 3 > (size_t)(INT32_MAX / 4)) return set_error(RT_E_INVALID, "photon map too large");
  std::set<rt_scene*> done;
  for (int q = 0; q < n; ++q) {
    if (!done.insert(scenes[q]).second) continue;
    std::vector<double> p = fullPos, w = fullPwr;  // set_photon_map consumes its lists
    scenes[q]->photonsUploaded = false;
    if ((rc = set_photon_map(scenes[q], p, w))) return rc;
  }
  return RT_OK;
}

}  // extern "C"
