// VALU issue-cost probe (VERDICT r05 Next #2): SIMD cycles per wave64 instruction for each class in
// the render kernel's VALU mix (profiles/r05zf_c3_valu_mix.txt), at 1, 2 and 4 waves per SIMD.
//
// Every lane runs K = 16 independent instances of one instruction per loop trip (inline asm, so the
// compiler neither folds nor re-schedules them), enough in flight to cover the result latency at one
// wave per SIMD. Each wave times itself with s_memtime (a shader-clock tick, MI355X_MICROARCH.md
// "Per-instruction cycle constants") around the loop; with w waves resident on a SIMD the SIMD's cost
// of one instruction is  wave cycles / (instructions per wave x w).  The grid is exactly one 256-thread
// block (4 waves, one per SIMD) per CU per w, so every SIMD holds w waves for the whole loop.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_issue.hip -o tools/valu_issue && tools/valu_issue
// Prints one JSON object: {class: {"w1": cyc, "w2": cyc, "w4": cyc, "winst_per_ns_per_simd": r, "ms": t}, ...}.
// Where the waves of a w-launch do not all overlap (dispatch ramp, uneven blocks per CU) the w-columns
// understate the cost; the event-timed rate (8 waves per SIMD, 8 rounds) does not depend on that.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int K = 16;
constexpr int ITERS = 2048;

enum Op {
  FMA_F64, ADD_F64, MUL_F64, MIN_F64, MAX_F64, CMP_F64_SGPR, CMP_F64_VCC, CNDMASK_B32, MOV_B32, MOV_B64,
  ADD_U32, LSHL_B32, AND_B32, LSHL_B64, ADD_CO_U32, MBCNT, READFIRSTLANE, DPP_MOV, ADD_F32, FMA_F32, MAX3_F32,
  PK_ADD_F32, PK_FMA_F32, CVT_F32_F64, CMP_F32_SGPR, RCP_F64, FRACT_F64,
  CNDMASK_VCC, CMP_U32_VCC, CMP_CLASS_F64, OR_B32, LSHR_B32_VOP2, BFE_U32, MUL_LO_U32, CVT_F64_I32, LDEXP_F64,
  WRITELANE, SUB_U32, MAX_I32, NOP_OPS
};
static const char* kNames[NOP_OPS] = {
    "v_fma_f64", "v_add_f64", "v_mul_f64", "v_min_f64", "v_max_f64", "v_cmp_lt_f64_e64(sgpr)",
    "v_cmp_lt_f64(vcc)", "v_cndmask_b32_e64", "v_mov_b32", "v_mov_b64", "v_add_u32", "v_lshlrev_b32",
    "v_and_b32", "v_lshlrev_b64", "v_add_co_u32", "v_mbcnt_lo_u32_b32", "v_readfirstlane_b32", "v_mov_b32_dpp",
    "v_add_f32", "v_fma_f32", "v_max3_f32", "v_pk_add_f32", "v_pk_fma_f32", "v_cvt_f32_f64",
    "v_cmp_lt_f32_e64(sgpr)", "v_rcp_f64", "v_fract_f64",
    "v_cndmask_b32_e32(vcc)", "v_cmp_lt_u32(vcc)", "v_cmp_class_f64(vcc)", "v_or_b32", "v_lshrrev_b32(vgpr)",
    "v_bfe_u32", "v_mul_lo_u32", "v_cvt_f64_i32", "v_ldexp_f64", "v_writelane_b32", "v_sub_u32", "v_max_i32"};

template <int OP>
__device__ __forceinline__ void body(double* d, uint32_t* u, uint64_t* m, float* f, double dy, double dz, uint32_t uy,
                                     uint64_t mask, float fy, float fz) {
#pragma unroll
  for (int i = 0; i < K; ++i) {
    if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(dy), "v"(dz));
    if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dy));
    if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dy));
    if constexpr (OP == MIN_F64) asm volatile("v_min_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dy));
    if constexpr (OP == MAX_F64) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dy));
    if constexpr (OP == CMP_F64_SGPR) asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "=s"(m[i & 3]) : "v"(d[i]), "v"(dy));
    if constexpr (OP == CMP_F64_VCC) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(d[i]), "v"(dy) : "vcc");
    if constexpr (OP == CNDMASK_B32) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(uy), "s"(mask));
    if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i + 1) % K]));
    if constexpr (OP == MOV_B64) asm volatile("v_mov_b64 %0, %1" : "=v"(d[i]) : "v"(d[(i + 1) % K]));
    if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == LSHL_B32) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(u[i]));
    if constexpr (OP == AND_B32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == LSHL_B64) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(m[i]) : "v"(uy));
    if constexpr (OP == ADD_CO_U32) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(u[i]) : "v"(uy) : "vcc");
    if constexpr (OP == MBCNT) asm volatile("v_mbcnt_lo_u32_b32 %0, -1, %0" : "+v"(u[i]));
    if constexpr (OP == READFIRSTLANE) { uint32_t r_; asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(r_) : "v"(u[i])); }
    if constexpr (OP == DPP_MOV) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0" : "=v"(u[i]) : "v"(u[(i + 1) % K]));
    if constexpr (OP == ADD_F32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fy));
    if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fy), "v"(fz));
    if constexpr (OP == MAX3_F32) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fy), "v"(fz));
    if constexpr (OP == PK_ADD_F32) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[i]) : "v"(dy));
    if constexpr (OP == PK_FMA_F32) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[i]) : "v"(dy), "v"(dz));
    if constexpr (OP == CVT_F32_F64) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));
    if constexpr (OP == CMP_F32_SGPR) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m[i & 3]) : "v"(f[i]), "v"(fy));
    if constexpr (OP == RCP_F64) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
    if constexpr (OP == FRACT_F64) asm volatile("v_fract_f64 %0, %0" : "+v"(d[i]));
    if constexpr (OP == CNDMASK_VCC) asm volatile("s_mov_b64 vcc, %1\n\tv_cndmask_b32 %0, %0, %2, vcc" : "+v"(u[i]) : "s"(mask), "v"(uy) : "vcc");
    if constexpr (OP == CMP_U32_VCC) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(u[i]), "v"(uy) : "vcc");
    if constexpr (OP == CMP_CLASS_F64) asm volatile("v_cmp_class_f64 vcc, %0, %1" : : "v"(d[i]), "v"(uy) : "vcc");
    if constexpr (OP == OR_B32) asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == LSHR_B32_VOP2) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == BFE_U32) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(u[i]));
    if constexpr (OP == MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == CVT_F64_I32) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
    if constexpr (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[i]) : "v"(uy));
    if constexpr (OP == WRITELANE) asm volatile("v_writelane_b32 %0, %1, 5" : "+v"(u[i]) : "s"((uint32_t)mask));
    if constexpr (OP == SUB_U32) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
    if constexpr (OP == MAX_I32) asm volatile("v_max_i32 %0, %0, %1" : "+v"(u[i]) : "v"(uy));
  }
}

template <int OP>
__global__ void __launch_bounds__(256) probe(uint64_t* cyc, double* sink, double dy, uint32_t uy, float fy) {
  double d[K];
  uint32_t u[K];
  uint64_t m[K];
  float f[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    d[i] = 1.0 + threadIdx.x * 1e-7 + i;
    u[i] = threadIdx.x + i;
    m[i] = (uint64_t)threadIdx.x * 3 + i;
    f[i] = 1.0f + i;
  }
  const uint64_t mask = 0xAAAAAAAAAAAAAAAAull;
  const uint64_t t0 = clock64();
  const double dz = dy * 0.5;
  const float fz = fy * 0.25f;
  for (int it = 0; it < ITERS; ++it) body<OP>(d, u, m, f, dy, dz, uy, mask, fy, fz);
  const uint64_t t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) s += d[i] + u[i] + (double)m[i] + f[i];
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
  if (s == -1.2345) sink[0] = s;  // keeps every chain live; never true for these inputs
}

// per class: s_memtime cycles per instruction of the median wave at 1 / 2 / 4 resident waves per SIMD
// ("w1".."w4"), and the event-timed chip throughput with 8 waves per SIMD over 8 rounds of blocks:
// wave instructions per second per SIMD ("winst_per_ns_per_simd"); cycles at a clock f are f / that.
template <int OP>
void run(int cus, uint64_t* dcyc, double* dsink, FILE* o, bool last) {
  fprintf(o, "  \"%s\": {", kNames[OP]);
  for (int w : {1, 2, 4}) {
    const int blocks = cus * w;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, dcyc, dsink, 0.999, 3u, 0.5f);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> c((size_t)blocks * 4);
    (void)hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double med = (double)c[c.size() / 2];
    fprintf(o, "\"w%d\": %.3f, ", w, med / ((double)ITERS * K * w));
  }
  const int blocks = cus * 8 * 8;  // 8 waves per SIMD resident x 8 rounds
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, dcyc, dsink, 0.999, 3u, 0.5f);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, dcyc, dsink, 0.999, 3u, 0.5f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double winst = (double)blocks * 4 * ITERS * K;
  fprintf(o, "\"winst_per_ns_per_simd\": %.5f, \"ms\": %.3f}%s\n", winst / (ms * 1e6) / (cus * 4.0), ms, last ? "" : ",");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

template <int... OPS>
void run_all(int cus, uint64_t* dcyc, double* dsink, std::integer_sequence<int, OPS...>) {
  (run<OPS>(cus, dcyc, dsink, stdout, OPS == NOP_OPS - 1), ...);
}

int main() {
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) != hipSuccess) { printf("{\"error\": \"no device\"}\n"); return 1; }
  const int cus = pr.multiProcessorCount;
  uint64_t* dcyc;
  double* dsink;
  if (hipMalloc(&dcyc, sizeof(uint64_t) * cus * 4 * 64) != hipSuccess || hipMalloc(&dsink, 8) != hipSuccess) return 1;
  printf("{\"probe\": \"valu_issue\", \"cus\": %d, \"unroll\": %d, \"iters\": %d, "
         "\"unit\": \"SIMD cycles per wave64 instruction (s_memtime), median wave\",\n \"classes\": {\n", cus, K, ITERS);
  run_all(cus, dcyc, dsink, std::make_integer_sequence<int, NOP_OPS>{});
  printf(" }}\n");
  (void)hipFree(dcyc);
  (void)hipFree(dsink);
  return 0;
}
