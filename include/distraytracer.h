/*
 * distraytracer.h -- C ABI of the MI355X-native trace loop (libdistraytracer.so).
 *
 * Drop-in boundary for the reference's render entry, the abstract
 * `myScene.draw()` (src/rayTracerDistAccelShdPhtnMap/myScene.java:1182),
 * implemented by `myFOVScene.draw()` (myScene.java:1481-1531) and reached from
 * the `.cli` `write` command (myRTFileReader.java:86-93) and from
 * `DistRayTracer.draw()` (DistRayTracer.java:77). Everything below that call
 * -- shootMultiRays (:1447), reflectRay (:907), findClosestRayHit (:888),
 * calcShadow (:879), the myGeomBase/myBVH traversal (myGeomBase.java:132-421),
 * myObjShader.getColorAtPos (myObjShader.java:409) and the photon kNN gather
 * (myLight.java:389-445) -- runs as HIP kernels on gfx950.
 *
 * Two ways in:
 *   rt_scene_create(desc)  the flattened myScene the Java side would hand over
 *                          through JNI (objList/lightList/shaders/CTMs/accel
 *                          groups; INTEGRATION.md shows the binding);
 *   rt_scene_load_cli()    the native mirror of myRTFileReader.readRTFile
 *                          (myRTFileReader.java:15-349) that builds that same
 *                          desc from a `.cli` file, then calls rt_scene_create.
 *
 * Conventions: every function returns 0 on success or a negative RT_E* code;
 * rt_last_error() gives a thread-local message. No exceptions or longjmp cross
 * the ABI. Output buffers are caller-owned and never retained. One in-flight
 * render per scene; distinct scenes may render concurrently. Products of this
 * library are GPU-only: there is no CPU fallback (RT_E_NODEVICE when no GPU).
 */
#ifndef DISTRAYTRACER_H
#define DISTRAYTRACER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 7

enum rt_status {
  RT_OK = 0,
  RT_E_INVALID = -1,  /* bad argument / malformed desc */
  RT_E_PARSE = -2,    /* .cli parse error or unsupported command */
  RT_E_IO = -3,       /* file not found */
  RT_E_NODEVICE = -4, /* no HIP device */
  RT_E_HIP = -5,      /* HIP runtime error */
  RT_E_OOM = -6
};

/* primitive kinds (objType.java; readPrimData myScene.java:447-521) */
enum rt_prim_type {
  RT_PRIM_TRIANGLE = 0,  /* myTriangle */
  RT_PRIM_QUAD = 1,      /* myQuad */
  RT_PRIM_PLANE = 2,     /* myPlane (infinite) */
  RT_PRIM_SPHERE = 3,    /* mySphere / ellipsoid / sphereIn */
  RT_PRIM_MOVING_SPHERE = 4,
  RT_PRIM_CYLINDER = 5,  /* myCylinder (capped) */
  RT_PRIM_HOLLOW_CYLINDER = 6,
  RT_PRIM_BOX = 7        /* myRndrdBox */
};
#define RT_PRIM_INVERTED 1 /* sphereIn: normals point in (mySceneObject.invertedIDX) */

typedef struct rt_prim_desc {
  int32_t type;     /* rt_prim_type */
  int32_t material; /* index into rt_scene_desc.materials */
  int32_t flags;    /* RT_PRIM_INVERTED */
  int32_t nverts;   /* planar: 3 or 4 */
  double ctm[16];   /* row-major CTM: matrix-stack top when the object was created */
  double v[4][3];   /* planar vertices in file order */
  double uv[4][2];  /* texture_coord per vertex */
  /* sphere: cx cy cz rx ry rz [x1 y1 z1 for moving]; cylinder: r h cx cy cz ox oy oz;
     box: xmin ymin zmin xmax ymax zmax; plane: a b c d */
  double p[12];
} rt_prim_desc;

/* myScene.txtrType (myScene.java:117, getCurTexture :531-542) */
enum rt_texture_kind { RT_TEX_NONE = 0, RT_TEX_IMAGE = 1, RT_TEX_NOISE = 2, RT_TEX_WOOD = 3, RT_TEX_MARBLE = 4,
                       RT_TEX_STONE = 5, RT_TEX_WOOD2 = 6 };
#define RT_MAX_NOISE_COLORS 16

typedef struct rt_material_desc { /* myObjShader.setCurrColors (myObjShader.java:51-75) */
  int32_t simple;       /* 1 = mySimpleReflObjShdr (`shiny` with ktrans/index) */
  int32_t texture;      /* rt_texture_kind */
  int32_t tex_top;      /* texture index for RT_TEX_IMAGE "top", -1 none */
  int32_t use_photon_map, caustic_photons;
  int32_t octaves, rnd_colors, use_fwd_trans;
  double diffuse[3], ambient[3], specular[3]; /* already clamped <= 1 (myColor) */
  double phong_exp, k_refl, k_refl_clr[3], k_trans, perm, perm_clr[3];
  double noise_scale, turb_mult, color_scale, color_mult, period_mult[3];
  double colors[RT_MAX_NOISE_COLORS][3]; /* noise colours (noise_color list or the texture's defaults) */
  int32_t num_colors;
  /* RT_TEX_STONE (myCellularTexture): 0 Manhattan / 1 Euclid, ROI function 0..8, points per ROI */
  int32_t dist_func, roi_func, num_pts_dist;
  double avg_per_cell, mortar_thresh;
} rt_material_desc;

enum rt_light_type { RT_LIGHT_POINT = 0, RT_LIGHT_SPOT = 1, RT_LIGHT_DISK = 2 };
typedef struct rt_light_desc { /* myLight.java */
  int32_t type, pad;
  double pos[3], color[3], dir[3];
  double inner_deg, outer_deg, radius;
  double ctm[16];
} rt_light_desc;

typedef struct rt_accel_desc { /* myScene.endTmpObjList (myScene.java:305-324) */
  int32_t type;        /* 0 = end_list (myGeomList), 1 = end_accel (myBVH) */
  int32_t first, count; /* range of rt_scene_desc.accel_members (prim indices or RT_INSTANCE_REF, tmp-list order) */
  int32_t pad;
  double ctm[16];      /* CTM when end_list/end_accel ran */
} rt_accel_desc;

/* myInstance (mySceneObject.java:95-145): `instance <name> [shdr]` of a `named_object`
   (myScene.java:378-395), also the elements `sierpinski` lays out (myScene.java:339-377). */
typedef struct rt_instance_desc {
  int32_t base;      /* the named object: >= 0 prim index, < 0 ~accel index (an accel holding no instances) */
  int32_t material;  /* instance shader (useInstShader), -1: the object's own shaders */
  double ctm[16];    /* row-major: named object's CTM x matrix-stack top (buildCTMara, DistRayTracer.java:401) */
  double origin[3];  /* trans_origin: matrix-stack top x (0,0,0) (myGeomBase ctor, myGeomBase.java:39) */
} rt_instance_desc;
/* rt_scene_desc.top / accel_members entry naming instance i */
#define RT_REF_INSTANCE 0x40000000
#define RT_INSTANCE_REF(i) (RT_REF_INSTANCE | (int32_t)(i))

typedef struct rt_texture_desc {
  int32_t w, h;
  const uint8_t* rgb; /* w*h*3 RGB8, row-major, row 0 = top (Processing PImage order) */
} rt_texture_desc;

typedef struct rt_scene_desc {
  int32_t num_prims;
  const rt_prim_desc* prims; /* every renderable primitive, creation order (= RNG prim key) */
  int32_t num_materials;
  const rt_material_desc* materials;
  int32_t num_lights;
  const rt_light_desc* lights; /* lightList order */
  int32_t num_accels;
  const rt_accel_desc* accels;
  const int32_t* accel_members;
  int32_t num_top;
  const int32_t* top; /* objList order: >= 0 prim index (or RT_INSTANCE_REF), < 0 accel ~index */
  int32_t num_textures;
  const rt_texture_desc* textures;
  double fov;            /* degrees */
  double background[3];
  int32_t bkg_texture;   /* -1 none; else skydome texture index */
  int32_t rays_per_pixel;
  double skydome[4];     /* radius, cx, cy, cz */
  int32_t dof;           /* lens set: depth of field (FOV camera only, myFOVScene.draw) */
  int32_t camera;        /* RT_CAMERA_*: the scene subclass the .cli selected (myRTFileReader.java:51-83) */
  double lens_radius, lens_focal;
  int32_t photon_mode;   /* 0 none, 1 diffuse_photons, 2 caustic_photons */
  int32_t photon_count, photon_k, pad1;
  double photon_max_dist; /* already rounded through float (Float.parseFloat) */
  double camera_param[2];  /* RT_CAMERA_FISHEYE: {aperture degrees, 0}; RT_CAMERA_ORTHO: {width, height} */
  int32_t num_instances, pad2;
  const rt_instance_desc* instances;
} rt_scene_desc;

/* rt_scene_desc.camera */
enum { RT_CAMERA_FOV = 0, RT_CAMERA_FISHEYE = 1, RT_CAMERA_ORTHO = 2 };

typedef struct rt_render_params {
  int32_t width, height; /* image size (the reference hard-codes 300x300, DistRayTracer.java:15-16) */
  int32_t spp;           /* <= 0: the scene's rays_per_pixel */
  int32_t row0, row1;    /* rows [row0,row1) of the image; row1 <= 0 means height */
  int32_t row_step;      /* <= 1: every row; >1: interleaved bands (multi-GPU) */
  uint64_t seed;         /* keyed RNG seed */
  uint32_t flags;        /* RT_RENDER_* */
  int32_t row_band;      /* <= 1: single rows. The rendered rows are row0 + k*row_step*row_band + j,
                            0 <= j < row_band, below row1; output row i is the i-th of them */
} rt_render_params;

/* rt_render_params.flags: run the all-features kernel instead of the one specialised
   to the scene's features (results are identical; for testing the specialisation) */
#define RT_RENDER_GENERIC 1u
/* dispatch tiles in row-major order instead of the probed longest-first schedule
   (results are identical; for testing and timing the schedule) */
#define RT_RENDER_ROWMAJOR 2u
/* test every top-level primitive (no bounding-sphere culling): same image, slower */
#define RT_RENDER_NOCULL 4u
/* trace the shadow rays of a wave's shading step compacted (ballot + prefix count: lane e traces
   the e-th (hit, light) pair) instead of light by light on the shading lanes: same image (DESIGN.md
   §4 "Compacted shadow rays"; slower on the benchmark configs, so not the default). It packs a
   lane's RNG key into 64 bits, so it needs width * height <= 2^32 and spp < 2^20 (RT_E_INVALID
   otherwise); renders without the flag have no such limit */
#define RT_RENDER_SHCOMPACT 8u
/* turn off the wave-level candidate test of shadow rays against the top-level entries' bounding
   spheres (DESIGN.md §4 "Wave-level shadow cull"): same image; for A/B timing and testing */
#define RT_RENDER_NOWAVECULL 16u
/* level-synchronous shading (DESIGN.md §4 "Level-synchronous shading"): each generation of the shading
   tree is one launch over a compacted ray queue, frames in HBM records, folded bottom up; same image.
   Blocks until the frame is done (it reads each level's ray count); not with tile lists. */
#define RT_RENDER_WAVEFRONT 32u
/* one pixel per wave (64 sample lanes; lanes past spp idle) instead of 64 / G pixels of G samples:
   same samples, same per-pixel order, same image; a layout of width x height one-pixel tiles */
#define RT_RENDER_PIXEL_WAVES 64u

typedef struct rt_scene rt_scene;

/* counters (RT_ST_*) reported by rt_render_count */
enum {
  RT_ST_CAMERA = 0, RT_ST_SHADOW, RT_ST_REFL, RT_ST_REFR, RT_ST_BOX, RT_ST_TRI, RT_ST_QUAD, RT_ST_IMPLICIT,
  RT_ST_LIGHT, RT_ST_PHOTON, RT_ST_TEXEL, RT_ST_NODE, RT_ST_LEAF, RT_ST_MEMBER, RT_ST_ROOT, RT_ST_TOP,
  /* the same record loads counted per WAVE step for records a wave loads once for all its
     lanes (packet traversal, wave-uniform top-level entries and lights); per lane elsewhere */
  RT_ST_W_NODE, RT_ST_W_TRI, RT_ST_W_QUAD, RT_ST_W_IMPLICIT, RT_ST_W_LIGHT, RT_ST_W_PHOTON,
  RT_ST_N = 24
};

int rt_abi_version(void);
/* Provenance (ABI 5): a hash of the sources, headers and compiler flags this library was built
   from (distraytracer_old_amd/build.py build_id); profiles and bench lines record it. */
const char* rt_build_id(void);
const char* rt_last_error(void);
int rt_device_count(int* count);

int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out);
int rt_scene_load_cli(const char* scene_dir, const char* cli_file, int num_textures, const char* const* texture_names,
                      const rt_texture_desc* textures, int device, rt_scene** out);
/* Host-only parse + build (no device): fills the rt_scene_info fields; device bytes = layout bytes. */
int rt_scene_inspect_cli(const char* scene_dir, const char* cli_file, int num_textures, const char* const* texture_names,
                         const rt_texture_desc* textures, int64_t* info, int n);
/* info[0..13]: objects, lights, bvh_internal, bvh_leaves, bvh_depth, bvh_prims, prims, rays_per_pixel,
   device bytes, triangles, photons (stored), materials, photon mode (0 none / 1 diffuse / 2 caustic),
   photons emitted per light */
int rt_scene_info(const rt_scene* scene, int64_t* info, int n);
/* PNG name myScene.saveFile gives the image (myScene.java:1185-1196): the `write` argument
   (myRTFileReader.java:86-88; the .cli file name when the file has none) with its last
   extension removed, plus ".png". rt_png_name applies the rule to any name; rt_scene_save_name
   to the name recorded by rt_scene_load_cli (RT_E_INVALID for a scene built from a desc).
   Both return the name's length, writing it NUL-terminated when it fits in cap. */
int rt_png_name(const char* save_name, char* buf, int cap);
int rt_scene_save_name(const rt_scene* scene, char* buf, int cap);
void rt_scene_destroy(rt_scene* scene);

/* photon-map pre-pass (myScene.initRender :1096-1099); idempotent per scene. The kNN gather of
   the render reads DISTRAYTRACER_KNN_U16_MAX (0..65535, default 65535) at rt_scene_create /
   rt_scene_load_cli: the photons per counting pass its 16-bit buckets take before a lane
   repeats the pass with 32-bit ones -- a testing knob; the image does not depend on it. */
int rt_photons_build(rt_scene* scene, uint64_t seed);
/* The photon map built by rt_photons_build as the reference's photon_list (myScene.java:1000-1091,
   insertion order): *count = number of photons; copies min(n, count) positions / powers
   (double[3] each) to pos / pwr. */
int rt_scene_photons(const rt_scene* scene, double* pos, double* pwr, int64_t n, int64_t* count);
/* The photon map's search structure as the device holds it (inspection / tests): *n_nodes = its
   node count (NodeD records of 128 bytes, csrc/rt_types.h), *root = the root node; copies up to
   node_cap records to nodes and up to n leaf-ordered positions / powers (double[3]) to ppos / ppwr
   (any of them may be NULL). Built on the GPU (photon_build.hip) or, for a map of one leaf or with
   DISTRAYTRACER_PHOTON_BUILD=host in the environment, on the host (photon.cpp): the same structure. */
int rt_scene_photon_map(const rt_scene* scene, void* nodes, int64_t node_cap, double* ppos, double* ppwr, int64_t n,
                        int64_t* n_nodes, int32_t* root);
/* Sharded pre-pass (multi-GPU): shoot only emitted photons [first, first+count) of
   every light (same keyed RNG, so the union of shards is the full pre-pass); the scene's
   photon_list becomes that shard (light-major, then photon index, then path order) without a
   search structure; per_light[num_lights] (may be NULL) receives the shard's count per light. */
int rt_photons_shoot(rt_scene* scene, uint64_t seed, int64_t first, int64_t count, int64_t* per_light);
/* Set the photon_list (insertion order) and build / upload the photon map from it. */
int rt_photons_set(rt_scene* scene, const double* pos, const double* pwr, int64_t n);

/* Blocking render into caller-owned HOST buffers (either may be NULL). Runs on the scene's own
   stream with device output buffers kept across calls (no per-call allocation or device-wide sync;
   they grow to the largest frame rendered and are freed by rt_scene_destroy).
   rgb: float[n_rows*width*3] clamped <=1 per myColor; argb: int32[n_rows*width], reference packing. */
int rt_render(rt_scene* scene, const rt_render_params* p, float* rgb, int32_t* argb);
/* Asynchronous render into caller-owned DEVICE buffers on `hip_stream` (hipStream_t, may be NULL).
   Tile dispatch order (never the pixels): the first render of a row layout orders tiles by a probe
   and records its waves' durations; the next render of that layout synchronises once and orders the
   tiles by those measured times (longest first). Render a layout twice before timing it. */
int rt_render_device(rt_scene* scene, const rt_render_params* p, float* d_rgb, int32_t* d_argb, void* hip_stream);
/* Tile partitions (multi-GPU). A render layout (p's size, rows and spp) is cut into
   wave tiles of tw x th pixels, numbered row-major over tiles_x columns of tiles.
   rt_tile_layout: out[0..3] = {ntiles, tiles_x, tw, th}.
   rt_tile_costs: the measured wave time of every tile of the layout (calibrating the layout first if no
   render of it has measured its waves; synchronous) into cost[min(ntiles, cap)]; returns ntiles.
   Layouts under 2^16 pixels are not scheduled (row-major dispatch): every tile costs 1.
   rt_render_tiles_device: render only the tiles tiles[0..ntiles) (a HOST int32 list, each < the
   layout's ntiles, dispatched in that order; validated and copied to the device once per distinct
   list, the last 16 kept) asynchronously on hip_stream into DEVICE buffers of the WHOLE layout (rgb float[n_rows*width*3], argb int32[n_rows*width]; pixels of other tiles are not written).
   Pixels do not depend on which tiles a launch holds: a partition of the tiles over N launches (or N
   GPUs) reassembles to the 1-launch image bit for bit. */
int rt_tile_layout(rt_scene* scene, const rt_render_params* p, int32_t* out);
int rt_tile_costs(rt_scene* scene, const rt_render_params* p, uint32_t* cost, int cap);
int rt_render_tiles_device(rt_scene* scene, const rt_render_params* p, const int32_t* tiles, int ntiles, float* d_rgb,
                           int32_t* d_argb, void* hip_stream);
/* Render only the listed pixels (indices row * width + col of a whole-frame layout: p's rows must be
   the whole image) with ONE sample per wave -- each pixel's samples run in parallel on as many
   SIMDs -- and each pixel summed in sample order: the same pixels as the other renders, written into
   whole-frame DEVICE buffers (other pixels untouched); asynchronous on hip_stream. For the handful of
   pixels whose shared wave would outlast a GPU's share of a multi-GPU frame (multigpu.py). */
int rt_render_pixels_device(rt_scene* scene, const rt_render_params* p, const int32_t* pixels, int npix, float* d_rgb,
                            int32_t* d_argb, void* hip_stream);
/* Instrumented render of the listed tiles (rt_render_count's counters for those tiles only; blocking). */
int rt_render_tiles_count(rt_scene* scene, const rt_render_params* p, const int32_t* tiles, int ntiles, uint64_t* stats);
/* `refine on` (myScene.setRefine, myScene.java:796-803): the progressive steps of a width x height
   render, largest first and ending at 1 (e.g. 16 8 4 2 1 at 300x300); returns their number n and
   copies min(n, cap) of them; n = 1 (steps {1}) when the scene does not refine. */
int rt_refine_steps(const rt_scene* scene, int width, int height, int* steps, int cap);
/* One refine pass of myFOVScene.draw (myScene.java:1481-1531; the other cameras alike): renders the
   pixels whose row and column are multiples of `step` and writes each over its step x step span
   (writePxlSpan, :1171-1177) into full-size HOST buffers rgb[height*width*3] / argb[height*width]
   (either may be NULL; other pixels are left untouched). skip_origin leaves pixel (0,0) alone (the
   reference skips it on every pass after the first). p's row fields are ignored. Pixel RNG keys are
   the full render's, so the passes 16, 8, ..., 1 end in rt_render's image. */
int rt_render_pass(rt_scene* scene, const rt_render_params* p, int step, int skip_origin, float* rgb, int32_t* argb);
/* Instrumented render (counters RT_ST_*: per lane, and RT_ST_W_* per wave step): same image,
   slower; stats: uint64[RT_ST_N] (24 since ABI 4). RT_RENDER_NOCULL in p->flags counts the
   reference algorithm's work (every objList entry tested). */
int rt_render_count(rt_scene* scene, const rt_render_params* p, float* rgb, int32_t* argb, uint64_t* stats);
/* The render-kernel instantiations a scene's renders use (ABI 6), as feature masks (the template
   argument F of render_kernel<CNT, F>, csrc/trace_kernels.h FT_*): *timed = the variant rt_render
   launches with `flags`, *counted = the counting variant rt_render_count launches -- the same mask for
   the benchmark configs' variants (C3 0, C4, C5), so the counted record loads are the timed kernel's. */
int rt_render_variant(const rt_scene* scene, uint32_t flags, uint32_t* timed, uint32_t* counted);
/* Kernel-only timing helper: average ms of the render kernel over `iters` launches (HIP events on the
   launch stream), inputs resident in HBM; at least 2 warmup launches (the schedule calibration). */
int rt_time_render(rt_scene* scene, const rt_render_params* p, int warmup, int iters, double* avg_ms);

/* ---- Multi-GPU frame (ABI 6) ---------------------------------------
   The reference's draw() (myScene.java:1481-1531) over N GPUs: the whole-frame layout's wave tiles,
   measured once on rank 0 (rt_tile_costs), are cut into N contiguous runs of equal cost, and the
   tiles whose own wave would outlast a rank's share are rendered one sample per wave beside them
   (rt_rank_plan). Every frame each rank renders its part into a device frame, ranks > 0 pack their
   pixels and send them to rank 0 (RCCL point-to-point over xGMI, grouped), and rank 0 -- which
   rendered its own part straight into the output frame -- scatters them in. Frame f's exchange
   overlaps frame f + 1's render (double-buffered slabs on a third stream per rank). The frame is
   bit-identical to rt_render's for every N and transport. */
typedef struct rt_group rt_group;
/* rt_group_create flags */
#define RT_GROUP_RGB 1u  /* exchange the float-RGB plane too (default: the ARGB ints, rndrdImg.pixels) */
#define RT_GROUP_COPY 2u /* transport: device / peer copies in this process instead of RCCL; ranks may
                            share a device (the one-GPU emulation of an N-GPU frame) */
/* The deterministic plan of a layout's tile costs (host only): owner[t] = the rank rendering tile t
   in its wave run, or world + rank when the tile is one of that rank's split (one sample per wave)
   tiles; order[0..ntiles) = every tile in dispatch order (longest first by quarter-octave cost
   bucket, row-major inside a bucket): a rank's run and split tiles are the subsequences of order it
   owns. heavy <= 0: 1.25 (a tile is split when its cost exceeds heavy x total / (slots x world));
   slots <= 0: 4096 (wave slots of one MI355X at the render kernel's occupancy). weight (may be NULL):
   per-tile factors of the cut (the runs hold equal sums of cost x weight; rt_group_rebalance); it must
   hold ntiles entries, like cost. */
int rt_rank_plan(const uint32_t* cost, const double* weight, int ntiles, int world, double heavy, int slots,
                 int32_t* owner, int32_t* order);
/* One process, n ranks: scenes[i] (rt_scene_create / rt_scene_load_cli on its device) is rank i.
   RCCL transport (ncclCommInitAll; one distinct device per rank) unless RT_GROUP_COPY. p: the frame
   (width, height, spp, seed, flags; row fields ignored). Calibrates the layout on scenes[0]. */
int rt_group_create(rt_scene* const* scenes, int n, const rt_render_params* p, uint32_t flags, double heavy, int slots,
                    rt_group** out);
/* One process per GPU: this process is `rank` of `world` (collective: every rank calls it). unique_id:
   the 128 bytes rt_group_unique_id returned on rank 0, shared by the caller (e.g. over
   torch.distributed); rank 0 calibrates and broadcasts the tile costs over RCCL. The group makes and
   owns an RCCL communicator (rt_comm_create_rccl + rt_group_create_comm). */
int rt_group_unique_id(void* id, int cap);
int rt_group_create_rank(rt_scene* scene, int rank, int world, const void* unique_id, const rt_render_params* p,
                         uint32_t flags, double heavy, int slots, rt_group** out);
/* Enqueue one frame (asynchronous). d_rgb / d_argb: rank 0's output frame, device buffers on its
   device (rgb float[H*W*3] needs RT_GROUP_RGB; NULL: the group's own frame, rt_group_frame); ignored
   in processes without rank 0. rt_group_sync waits for every stream of the ranks this process drives. */
int rt_group_render(rt_group* g, float* d_rgb, int32_t* d_argb);
int rt_group_sync(rt_group* g);
/* Blocking frame into caller-owned HOST buffers (either may be NULL) on rank 0's process -- the JNI
   draw() over N GPUs; other processes render their part and return. */
int rt_group_render_host(rt_group* g, float* rgb, int32_t* argb);
int rt_group_frame(rt_group* g, float** d_rgb, int32_t** d_argb);
/* info[0..9]: world, ranks driven by this process, first of them, layout tiles, tiles_x, tw, th,
   transport (1 RCCL / 2 host comm / 0 copies or one rank), frames enqueued, plan checks passed
   (rank mode, world > 1: the collective plan agreement checks, one per cut) */
int rt_group_info(const rt_group* g, int64_t* info, int n);
/* the plan (rt_rank_plan's owner / order, up to cap tiles); returns the tile count */
int rt_group_plan(const rt_group* g, int32_t* owner, int32_t* order, int cap);
/* every pixel (row * width + col) rank `rank` writes, in the order it sends them (its run's tiles,
   then its split pixels); returns the count */
int rt_group_rank_pixels(const rt_group* g, int rank, int32_t* pixels, int64_t cap);
/* mean HIP-event time of a driven rank's render (run + split pixels) over its frames since the last
   call (up to the last 64); synchronises that rank's render stream */
int rt_group_kernel_ms(rt_group* g, int rank, double* avg_ms, int* frames);
/* One-process RT_GROUP_COPY groups: `rank`'s step alone, frames pipelined as rt_group_render does
   (render, pack, copy into rank 0's slab, the scatter of its slice; rank 0: render + the whole
   scatter): wall-clock ms per step and the mean HIP-event ms of its render (the N-GPU step's
   non-kernel cost, measured on one GPU) */
int rt_group_time_rank(rt_group* g, int rank, int warmup, int iters, double* step_ms, double* kernel_ms);
/* counters (rt_render_count's) of a driven rank's part: its run and its split tiles (counted as tile
   waves; blocking) */
int rt_group_count(rt_group* g, int rank, uint64_t* stats);
/* Re-cut the plan from measured rank render times, `rounds` times (collective in rank mode): each
   round times every rank's render over `iters` frames (one-process groups: one rank at a time), folds
   each rank's time per unit of predicted cost into its tiles' cut weights and cuts again (split
   tiles and dispatch order unchanged). rank_ms[world] (may be NULL): the ranks' render times measured
   after the last cut. */
int rt_group_rebalance(rt_group* g, int rounds, int iters, double* rank_ms);
void rt_group_destroy(rt_group* g);
/* ---- Communicators (ABI 7) ------------------------------------------------------------------------
   The transport a one-process-per-GPU group and the sharded photon pre-pass run their collectives
   over. Two kinds:
     RCCL  rt_comm_create_rccl: an RCCL communicator of `world` ranks (unique_id from
           rt_group_unique_id on rank 0, shared by the caller); the frame exchange is stream-ordered
           ncclSend / ncclRecv over xGMI. One device per rank (RCCL refuses two ranks on one device).
     host  rt_comm_create_host: the caller's own transport (e.g. Java sockets / MPI, or
           torch.distributed's gloo in the tests) as four blocking callbacks on HOST buffers; the frame
           exchange stages the packed pixels through pinned host memory. Ranks may share a device, so
           an N-rank frame runs as N processes on one GPU -- the same rank-mode code path as RCCL
           (cost broadcast, plan check, receive offsets, rebalance all-gather), only the byte mover
           differs.
   Every collective of a group or of rt_photons_build_comm is entered by every rank in the same order
   with the same sizes; a rank's local failure travels as a status word inside that collective, so
   all ranks fail together instead of leaving peers blocked. A communicator must outlive the groups
   made from it and is used by one thread at a time. */
typedef struct rt_comm rt_comm;
typedef struct rt_comm_ops {
  void* ctx; /* passed back to every callback */
  /* each returns 0 on success (nonzero: the calling rt_* function returns RT_E_HIP) */
  int (*bcast)(void* ctx, void* buf, int64_t bytes, int root);               /* in place, from root */
  int (*allgather)(void* ctx, const void* in, void* out, int64_t bytes);     /* out[world * bytes], rank order */
  int (*send)(void* ctx, const void* buf, int64_t bytes, int peer);          /* blocking point-to-point */
  int (*recv)(void* ctx, void* buf, int64_t bytes, int peer);
} rt_comm_ops;
int rt_comm_create_rccl(int rank, int world, const void* unique_id, int device, rt_comm** out);
int rt_comm_create_host(int rank, int world, const rt_comm_ops* ops, rt_comm** out);
/* info[0..3]: rank, world, transport (1 RCCL / 2 host), device (-1 for host) */
int rt_comm_info(const rt_comm* comm, int64_t* info, int n);
void rt_comm_destroy(rt_comm* comm);
/* Diagnostics: the communicator's collectives on n int32 per rank, data checked on the host -- an
   all-gather, a broadcast from every rank, and (host transport) the group's exchange pattern: ranks
   > 0 send to rank 0 in rank order and rank 0 answers each. Collective; host-only for the host
   transport (no GPU needed), so the transport's bindings are testable on a CPU. */
int rt_comm_selftest(rt_comm* comm, int n);
/* rt_group_create_rank over a communicator (collective: every rank calls it). Rank 0 calibrates the
   layout and broadcasts the tile costs; before that the ranks check that they were given the same
   frame (size, spp, seed, flags, heavy, slots), and after every cut (here and in rt_group_rebalance)
   that they derived the same plan -- every sender's offset in rank 0's receive slab, pixel count and
   pixel-list hash against rank 0's receive side (rt_group_info plan_checks counts the checks passed).
   A NULL comm is a one-rank group. */
int rt_group_create_comm(rt_scene* scene, rt_comm* comm, const rt_render_params* p, uint32_t flags, double heavy,
                         int slots, rt_group** out);
/* The photon pre-pass (myScene.initRender, myScene.java:1096-1099) sharded over a communicator's
   ranks: rank r shoots emitted photons [r P / N, (r + 1) P / N) of every light
   (sendDiffusePhotons / sendCausticPhotons, myScene.java:952-1091, same keyed RNG), the shards are
   exchanged (each rank's records broadcast from it), merged into the reference's photon_list order
   (light-major, then photon index, then path order) and every rank builds the same photon map: the
   scene ends as rt_photons_build leaves it, bit for bit. Collective; NULL comm = rt_photons_build.
   rt_photons_build_local: the same over n scenes in one process (scenes[q] shoots shard q; scenes
   may repeat, e.g. n ranks emulated on one device); every distinct scene gets the merged map. */
int rt_photons_build_comm(rt_scene* scene, rt_comm* comm, uint64_t seed);
int rt_photons_build_local(rt_scene* const* scenes, int n, uint64_t seed);

/* Diagnostics: every RCCL entry point the group resolves at run time, called on `device` through a
   one-rank communicator -- ncclCommInitRank and ncclCommInitAll, ncclBroadcast, ncclAllGather and a
   grouped ncclSend / ncclRecv to itself of n int32 -- with the data checked on the host. A one-GPU
   machine cannot run two RCCL ranks (RCCL refuses two ranks on one device), so this is how the
   transport's bindings are exercised there. Returns RT_OK or an error. */
int rt_group_rccl_selftest(int device, int n);

/* Diagnostics: the device's fdlibm sin / cos / asin / acos (the sequences the trace kernels use,
   shared bit for bit with the CPU oracle) of x[0..n) into out[4*i .. 4*i+3], host buffers. */
int rt_math_eval(const double* x, double* out, int64_t n, int device);
/* Diagnostics: the render kernel's photon gather (getIrradianceFromPhtnTree, myObjShader.java:441-458)
   at points pts[3*i..3*i+2] into out[3*i..3*i+2] (host buffers); needs the scene's photon map. */
int rt_photon_gather(rt_scene* scene, const double* pts, double* out, int64_t n);
/* Host-only: the reference's photon kd-tree (myKD_Tree.build_tree, myLight.java:332-381) over a
   photon_list pos[3*n] (insertion order), as the device's tie replay uses it: out[4*i..4*i+3] =
   {photon (list index), split axis (-1: leaf), left, right} of node i, DFS pre-order, root 0. */
int rt_photon_kdtree(const double* pos, int64_t n, int32_t* out);
/* The scene's device copy of that kd-tree (n = photon count): out[4*i..4*i+3] = {photon as its index in
   the photon map's leaf-ordered arrays (rt_scene_photon_map ppos / ppwr), axis, left, right}. */
int rt_scene_photon_kdtree(const rt_scene* scene, int32_t* out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* DISTRAYTRACER_H */
