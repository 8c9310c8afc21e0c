// Internal host-side declarations shared by the loader, builder and HIP launch code.
#pragma once
#include <cstring>
#include <string>
#include <vector>

#include "../../include/distraytracer.h"
#include "rt_types.h"

namespace rt {

int set_error(int code, const std::string& msg);

// Quarter-octave bucket of a measured wave time (dispatch order key, longest first): 0 for 0, else
// 1 + floor(4 log2 c) by exact threshold compares (trace.hip sort_tiles, group.hip plan_ranks).
inline int cost_bucket(uint32_t c) {
  if (!c) return 0;
  const int oct = 31 - __builtin_clz(c);
  const double f = (double)c / (double)(1u << oct);  // [1, 2)
  return 1 + 4 * oct + (f >= 1.6817928305074290) + (f >= 1.4142135623730951) + (f >= 1.1892071150027210);
}

// Flattened scene on the host (mirrors SceneD) -- built by scene_build.cpp.
struct HostScene {
  std::vector<XformD> xf;
  std::vector<TriD> tri;
  std::vector<double> triUV;  // texture_coord of the 3 vertices (file order), 6 per triangle
  std::vector<PrimD> prim;
  std::vector<NodeD> node;
  std::vector<LeafD> leaf;
  std::vector<int32_t> member;
  std::vector<AccelD> accel;
  std::vector<TopD> top;
  std::vector<MatD> mat;
  std::vector<LightD> light;
  std::vector<TexD> tex;
  std::vector<uint32_t> texel;
  // photon map: BVH + leaf-ordered arrays (device layout) and the insertion-order list
  std::vector<NodeD> pnode;
  std::vector<double> ppos, ppwr;
  std::vector<double> photonListPos, photonListPwr;
  int photonRoot = 0;
  int64_t nphoton = 0;
  int64_t pnodeCount = 0;  // photon-map nodes (host- or device-built)
  // scene parameters
  double fov = 60;
  double bg[3] = {0, 0, 0};
  int bkgTex = -1;
  double sky[4] = {0, 0, 0, 0};
  int dof = 0;
  double lensRadius = 0, lensFocal = 0;
  int camera = 0;  // RT_CAMERA_*
  double cameraParam[2] = {0, 0};
  int rpp = 0;
  int photonMode = 0, photonCount = 0, photonK = 0;
  double photonMaxD2 = 0;
  // statistics (compare with the oracle's builder)
  int64_t bvhInternal = 0, bvhLeaves = 0, bvhDepth = 0, bvhPrims = 0, nprims = 0;
};

int build_host_scene(const rt_scene_desc* d, HostScene& hs);  // scene_build.cpp
// photon.cpp: photon-map search structure from the photon_list in insertion order
void build_photon_tree(HostScene& hs, const std::vector<double>& pos, const std::vector<double>& pwr);
// photon.cpp: the reference's kd-tree (myKD_Tree.build_tree) over photon_list indices, and its
// photons renumbered to the photon map's leaf order (leafToList[i] = list index of leaf slot i)
std::vector<KdNodeD> build_java_kdtree(const std::vector<double>& pos);
void kd_to_leaf_order(std::vector<KdNodeD>& kd, const std::vector<int32_t>& leafToList);

}  // namespace rt

struct rt_scene;
namespace rt {
// photon_build.hip: the same structure built on the scene's device (n > PHOTON_LEAF)
// (with the reference's kd-tree after the BVH records, built on the device too)
int build_photon_tree_gpu(rt_scene* s, const double* pos, const double* pwr, int64_t n);
// trace.hip: the render launches the multi-GPU group (group.hip) drives. prepare_render fills the
// kernel parameters of a render (rt_render_params checks, wave layout, camera constants);
// launch_tile_list renders a validated DEVICE tile list, launch_pixel_list a validated DEVICE pixel
// list one sample per wave (per-sample colours in smpCol[npix * spp * 3] / smpTr[npix * spp]);
// both asynchronous on `stream` (hipStream_t).
int prepare_render(rt_scene* s, const rt_render_params* p, ParamsD& P);
int launch_tile_list(rt_scene* s, const ParamsD& P, uint32_t flags, const int32_t* dtiles, int ntiles, float* rgb,
                     int32_t* argb, void* stream);
int launch_pixel_list(rt_scene* s, const ParamsD& P, uint32_t flags, const int32_t* dpix, int npix, double* smpCol,
                      uint8_t* smpTr, float* rgb, int32_t* argb, void* stream);
// trace.hip: the photon pre-pass pieces comm.hip's sharded builds (rt_photons_build_comm / _local)
// share with rt_photons_build: the scene's photon parameters checked; emitted photons [first,
// first+count) of every light shot into pos / pwr (photon_list order, perLight[L] their counts per
// light); the photon map built from a whole photon_list (pos / pwr are consumed)
int check_photon_params(const HostScene& h);
int shoot_photons(rt_scene* s, uint64_t seed, int64_t first, int64_t count, std::vector<double>& pos,
                  std::vector<double>& pwr, std::vector<int64_t>& perLight);
int set_photon_map(rt_scene* s, std::vector<double>& pos, std::vector<double>& pwr);
// group.hip: the deterministic rank plan (rt_rank_plan)
void plan_ranks(const uint32_t* cost, int n, int world, double heavy, int slots, int32_t* owner, int32_t* order,
                const double* weight = nullptr);
}  // namespace rt

struct rt_scene {
  rt::HostScene hs;
  std::string saveName;  // `write` argument (or the .cli name) when loaded by rt_scene_load_cli
  bool refine = false;   // `refine on` (rt_refine_steps / rt_render_pass)
  int device = 0;
  rt::SceneD dev{};
  std::vector<void*> allocs;
  size_t devBytes = 0;
  bool photonsUploaded = false;
  void* counters = nullptr;  // device uint64[RT_ST_N]
  // rt_render / rt_render_count (host buffers): output buffers kept across calls (grow-only)
  // and the scene's own non-blocking stream, so the blocking per-frame entry (the JNI
  // nativeRender path) pays no hipMalloc / hipFree / device-wide synchronisation per call
  float* outRgb = nullptr;
  int32_t* outArgb = nullptr;
  size_t outCap = 0;  // pixels
  void* stage = nullptr;  // pinned host staging of rt_render's read-back (hipHostMalloc, grow-only)
  size_t stageCap = 0;    // bytes
  void* stream = nullptr;  // hipStream_t
  const double* noCullBound = nullptr;  // device [ntop][4] of -1 (RT_RENDER_NOCULL)
  // tile schedules (longest tiles first) per tile layout (trace.hip `schedule`)
  struct TileSchedule {
    std::string key;
    int32_t* order;  // device int32[ntiles]: dispatch position -> tile
    uint32_t* cost;  // device uint32[ntiles]: probe cost, then one launch's measured wave times
    int ntiles;
    int state;       // 0 probe order; 1 a measuring launch was issued; 2 ordered by measured times
    void* measured = nullptr;  // hipEvent_t recorded after the measuring launch, on its stream
    int tilesX = 0;            // the layout's tiles per row (XCD superblocks)
  };
  std::vector<TileSchedule> schedules;
  struct TileList {  // rt_render_tiles_device / rt_render_pixels_device: a validated list and its device copy
    std::vector<int32_t> host;
    int32_t* dev = nullptr;
    int32_t maxv = -1;  // its largest entry: a reuse checks it against the new layout's bound
  };
  std::vector<TileList> tileLists;
  // RT_RENDER_WAVEFRONT buffers (grow-only): level-0 records, sample colours, traced flags, level
  // counters, two ray queues, the records of levels 1..7
  enum { WF_NODE0, WF_SCOL, WF_TRACED, WF_CNT, WF_Q0, WF_Q1, WF_NODE1, WF_N = WF_NODE1 + 7 };
  void* wf[WF_N] = {};
  // rt_render_pixels_device: per-sample colours and traced flags of the listed pixels (grow-only)
  void* smpCol = nullptr;
  void* smpTr = nullptr;
  size_t smpCap = 0;  // samples
  size_t wfCap[WF_N] = {};
};
