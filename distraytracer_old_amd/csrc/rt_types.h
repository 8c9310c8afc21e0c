// Flattened scene layout in HBM (host builder <-> HIP kernels).
// DESIGN.md "Data layout in HBM" documents every record and its byte size.
#pragma once
#include <stdint.h>

namespace rt {

// Per distinct CTM (deduplicated by value): forward, inverse (myMatrix.InvertMe
// cofactor algorithm, myVector.java:111-196) and adjoint = inverse^T
// (DistRayTracer.java:399-405). 384 B.
struct XformD {
  double g[16];
  double inv[16];
  double adj[16];
};

// Triangle, 128 B: vertices in object space, file order; orientation A normal
// (orientation B is exactly -n); plane D for both
// orientations (setEQ uses the current first vertex, myPlanarObject.java:90).
struct TriD {
  double v[3][3];
  double n[3];
  double dA, dB;
  int32_t xf;   // own CTM
  int32_t xfc;  // accel CTM x own CTM (reCalcCTMHitNorm, Q4), -1 at top level
  int32_t mat;
  uint32_t key; // creation index (RNG prim key)
};

enum : int32_t {
  PT_TRI = 0, PT_QUAD = 1, PT_PLANE = 2, PT_SPHERE = 3, PT_MSPHERE = 4, PT_CYL = 5, PT_HCYL = 6, PT_BOX = 7,
  PT_INST = 8  // myInstance: never tested itself (trace_kernels.h inst_closest / inst_any)
};
// PrimD.flags
enum : int32_t { PF_INVERTED = 1, PF_INST_ACCEL = 2 };

// Every other primitive, 256 B. Field use by type:
//  QUAD/PLANE: a[0..11] v[4][3], a[12..14] NA, a[15..17] NB, a[18] DA, a[19] DB, a[20..27] uv[4][2]
//  SPHERE/MSPHERE: a[0..2] origin (origin0), a[3..5] radii, a[6..8] origin1
//  CYL/HCYL: a[0..2] origin, a[3] radX, a[4] radZ, a[5] height, a[6] yTop, a[7] yBottom, a[8..15] caps
//  BOX: a[0..2] min, a[3..5] max
//  INST: xf = instance CTM, xfc = list CTM x instance CTM when inside an accel (else -1),
//        mat = instance shader or -1, pad[0] = named object (PF_INST_ACCEL: accel index,
//        else its tri/prim ref)
struct PrimD {
  int32_t type, xf, xfc, mat;
  uint32_t key;
  int32_t flags;  // bit0 inverted (sphereIn)
  int32_t pad[2];
  double a[28];
};

// BVH node with both child boxes (reference topology, myBVH.addObjList
// myGeomBase.java:360-386). child >= 0: node index; child < 0: leaf ~index. 128 B =
// two 64-B lines, one per child (box + reference): a descent step reads only the
// left child's line, an unwind step only the right child's.
struct NodeD {
  double lmin[3], lmax[3];
  int32_t left;
  int32_t pad[3];   // photon map: left child range (start, count), right child start;
                    // scene BVH: pad[1..2] = the left child's fat-edge bound (double, node_slack)
  double rmin[3], rmax[3];
  int32_t right;
  int32_t padR[3];  // photon map: right child count, photons in the subtree; scene BVH: padR[1..2]
                    // = the right child's fat-edge bound
};
static_assert(sizeof(NodeD) == 128, "NodeD is two 64-B lines");
// fp32 copy of a NodeD's child boxes for the conservative fp32 box pre-test of the packet traversals
// (trace_kernels.h box32): b = left min[3] max[3], right min[3] max[3] rounded to nearest; mag >= every
// |coordinate| of both boxes; sl / sr >= the children's fat-edge bounds (node_slack) -- +inf where a
// value does not fit a float (the pre-test then settles nothing and the fp64 tests decide)
struct NodeF {
  float b[12];
  float mag, sl, sr, pad;
};
static_assert(sizeof(NodeF) == 64, "NodeF is one 64-B line");
// fp32 record of a TriD for the conservative fp32 edge pre-test of the packet traversals
// (trace_kernels.h tri_f32_out): m[j] = e_j x n with e_j = v_j - v_{j-1}, c[j] = v_j . m[j], n and dA
// rounded to nearest; k >= 2^-17 max_j |m_j| max(1, |n|) and tm >= max(|v_j|, |dA|) rounded up --
// k = +inf where a value is not finite or does not fit a float (the pre-test then rejects nothing)
struct TriF {
  float m[3][3];
  float c[3];
  float n[3];
  float d;
  float k, tm;
  float pad[2];
};
static_assert(sizeof(TriF) == 80, "TriF");
struct LeafD {
  int32_t start, count;  // range in leaf member refs (>= 0 tri index, < 0 ~prim index)
};
// Child references (NodeD.left/right, AccelD.root): >= 0 node index; < 0: c = ~ref is a
// leaf, either a LeafD index (bit 30 clear) or, with LEAF_RUN_FLAG, a run of `count`
// consecutive triangles starting at `start` (scene_build.cpp pack_leaves).
static constexpr int32_t LEAF_RUN_FLAG = 1 << 30;
static constexpr int32_t LEAF_RUN_MAXCOUNT = 31;
static constexpr int32_t LEAF_RUN_MAXSTART = (1 << 25) - 1;
inline int32_t leaf_run_ref(int32_t start, int32_t count) { return ~(LEAF_RUN_FLAG | (start << 5) | count); }
// A myBVH or a myGeomList (one leaf holding the whole list).
struct AccelD {
  double bmin[3], bmax[3];  // root box (list box / BVH root box)
  int32_t xf;
  int32_t root;      // child ref: >= 0 node, < 0 ~leaf
  int32_t is_list;   // end_list
  int32_t flags;     // ACCEL_NEAREST: the nearest-first closest-hit traversal applies (scene_build.cpp)
};
// AccelD.flags: a BVH whose leaves are all triangle runs in the accel's own CTM, with a finite
// fat-edge bound for every node (trace_kernels.h accel_closest_nf)
enum : int32_t { ACCEL_NEAREST = 1 };
// A node child's fat-edge bound: every point the reference's triangle test accepts for a
// triangle below the child lies within this distance of the child's box (per axis; in the
// accel's object space)
inline double& node_slack(NodeD& n, int side) { return *reinterpret_cast<double*>(side ? &n.padR[1] : &n.pad[1]); }
enum : int32_t { TOP_TRI = 0, TOP_PRIM = 1, TOP_ACCEL = 2, TOP_INST = 3 };  // TOP_INST: idx = PT_INST prim
struct TopD {
  int32_t kind, idx, xf;
  uint32_t key;
};

struct MatD {
  double diffuse[3], ambient[3], specular[3];
  double kreflclr[3], permclr[3];
  double phtnDiffScl[3], phtnPermClr[3];
  double phong, krefl, ktrans, perm, diffConst, avgDiffClr;
  // noise / marble
  double scale, turbMult, colorScale, colorMult, pmMag;
  double periodMult[3];
  double colors[16][3];  // RT_MAX_NOISE_COLORS
  // myCellularTexture: Poisson point-count table (cumulative probability keys, ascending)
  double mortar, pdfKey[14];
  int32_t pdfVal[14], npdf, ncolors;
  int32_t distFunc, roiFunc, numPtsDist, pad0;
  int32_t simple, hasCaustic, usePhotonMap, isCausticPhtn;
  int32_t tex, texTop, octaves, rndColors;
  int32_t useFwdTrans, pad[3];
};

struct LightD {
  int32_t type, index, pad[2];
  double origin[3];   // object space (getOrigin)
  double color[3];    // clamped <= 1
  double orient[3];   // normalized
  double tangent[3];  // disk surfTangent / spot oPhAxis
  double innerRad, outerRad, radDiff, radius;
  double g[16];       // light CTM (forward)
};

struct TexD {
  int32_t w, h;
  int64_t off;  // offset into the texel buffer (uint32 0xAARRGGBB)
};

// Photon map (myKD_Tree of myPhoton, myLight.java:278-446) on the device: a BVH over the
// photons (NodeD records; child ref >= 0 node, -1 leaf whose photon range [start,
// start+count) is in pad[0..1] (left) / pad[2], padR[0] (right); <= 24 photons per leaf) with
// the photon positions and powers as double[3] arrays in leaf order (csrc/photon.cpp). The k-nearest set a query finds does not depend on the
// search structure, so this replaces the reference's one-photon-per-node kd-tree.
static constexpr int PHOTON_LEAF = 24;
// The reference's own photon search structure, myKD_Tree (myLight.java:300-381): one photon per
// node, the median of its range after a stable sort on the axis of largest extent. Kept only for
// the exact replay of find_near at a tied k-th distance (trace_kernels.h knn_java). Stored after the
// photon BVH's NodeD records in the same allocation; the root record's padR[2] holds its offset in
// NodeD records (0: none). photon: the photon's index in the leaf-ordered ppos / ppwr arrays.
struct KdNodeD {
  int32_t photon, axis, left, right;  // axis -1: a leaf; child -1: none
};
static_assert(sizeof(KdNodeD) == 16, "KdNodeD");
static constexpr int KD_PER_NODED = (int)(sizeof(NodeD) / sizeof(KdNodeD));

// device-side scene handle (all pointers are device pointers)
struct SceneD {
  const XformD* xf;
  const TriD* tri;
  const TriF* triF;     // [ntri] fp32 edge records (tri_f32_out)
  const double* triUV;  // [ntri][3][2] texture_coord, nullptr when no triangle is image-textured
  const PrimD* prim;
  const NodeD* node;
  const NodeF* nodeF;   // [nnode] fp32 boxes of the BVH nodes (box32)
  const LeafD* leaf;
  const int32_t* member;
  const AccelD* accel;
  const TopD* top;
  const double* topBound;  // [ntop][4]: world bounding sphere (centre, radius) of a top-level
                           // implicit primitive, radius < 0 = none (trace.hip top_bounds)
  const MatD* mat;
  const LightD* light;
  const TexD* tex;
  const uint32_t* texel;
  const NodeD* pnode;   // photon BVH
  const double* ppos;   // [nphoton][3], leaf order
  const double* ppwr;   // [nphoton][3]
  int32_t ntop, nlight, nphoton, photonRoot;
  int32_t photonK;
  int32_t knnU16Max;  // photons per kNN counting pass the u16 buckets take (trace_kernels.h knn_hist_pass)
  double photonMaxD2;
  double bg[3];
  int32_t bkgTex;
  double sky[4];
  int32_t dof;
  double lensRadius, lensFocal;
  int32_t numRays;  // recursion budget (myScene.numRays = 8)
  // bit 0 (SCENE_FAST_SLAB): every BVH box coordinate is 0 or in [2^-200, 2^200] (trace_device.h
  // qdiv); bit 1 (SCENE_NEAREST_FIRST): nearest-first BVH traversals where they apply, set per launch
  // (RT_RENDER_NOCULL keeps the reference order: its counters are the reference algorithm's work);
  // bit 2 (SCENE_WAVE_CULL): wave-level shadow candidates (shadow_cands), ntop <= 64, culling on.
  // One word rather than a new field: the kernels' argument layout stays as it was.
  int32_t fastSlab;
};
enum : int32_t { SCENE_FAST_SLAB = 1, SCENE_NEAREST_FIRST = 2, SCENE_WAVE_CULL = 4 };

struct ParamsD {
  int32_t W, H, spp, row0, nrows, rowStep;
  uint64_t seed;
  double viewZ;
  // wave layout: G lanes per pixel (power of two, G <= spp) trace samples j, j+G, ...;
  // 64/G pixels per wave as a tw x th tile
  int32_t G, tw, th, band;  // band: output row ri is image row row0 + (ri/band)*rowStep*band + ri%band
  const int32_t* order;     // tile dispatch order (longest first), nullptr = row-major
  uint32_t* tcost;          // non-null: each wave writes its duration (s_memrealtime ticks) to tcost[tile]
  // camera (RT_CAMERA_*) with its per-image constants (setImageSize, myScene.java:780-792)
  int32_t cam, colStep;  // colStep: every colStep-th column (a `refine` pass, rt_render_pass)
  double fishMult, xStart, yStart, aperHalf;  // fisheye
  double orthPerRow, orthPerCol;              // ortho
};

}  // namespace rt
