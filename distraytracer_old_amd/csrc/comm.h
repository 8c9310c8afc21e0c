// Communicators (rt_comm_*, include/distraytracer.h ABI 7): the transport a one-process-per-GPU
// group (group.hip) and the sharded photon pre-pass (comm.hip) run their collectives over.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <string>

#include "rt_internal.h"

namespace rt {

// RCCL, resolved at run time (dlopen of librccl.so.1: in a PyTorch process the copy torch already
// loaded), so the library and the host transport work without it.
struct RcclApi {
  bool tried = false, ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclBroadcast) bcast = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclGetErrorString) errStr = nullptr;
};
extern RcclApi g_rccl;
int rccl_load();  // RT_OK or RT_E_INVALID (with the reason)

// Host-buffer collectives over either transport (RCCL stages through the communicator's device on
// its own stream and synchronises). Blocking; every rank calls the same sequence with the same sizes.
int comm_bcast(rt_comm* c, void* buf, size_t bytes, int root);
int comm_allgather(rt_comm* c, const void* in, void* out, size_t bytes);
// Point-to-point on host buffers: the host transport only (RCCL's are stream-ordered, group.hip).
int comm_send(rt_comm* c, const void* buf, size_t bytes, int peer);
int comm_recv(rt_comm* c, void* buf, size_t bytes, int peer);

// Every rank's `ok` (its local status before a collective step) combined: RT_OK when all ranks were
// ok, else an error naming the first failing rank (its own message when it is this rank).
int comm_all_ok(rt_comm* c, int local_rc, const char* what);

// Restores the caller's current HIP device on scope exit (the rt_group_* / rt_comm_* entry points
// switch devices while they work).
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace rt

struct rt_comm {
  int rank = 0, world = 1;
  bool rccl = false;
  int device = -1;  // RCCL: the communicator's device
  ncclComm_t nccl = nullptr;
  rt_comm_ops ops{};  // host transport
  hipStream_t st = nullptr;  // RCCL host-buffer collectives: staging stream and buffer (grow-only)
  void* dbuf = nullptr;
  size_t dcap = 0;
};
