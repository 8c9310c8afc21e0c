// C3's (triangles only) and C5's (photon map) render-kernel variants, compiled with the
// register-minimising machine scheduler (build.py SOURCE_FLAGS); trace.hip launches them
// through the host stubs this file instantiates (extern template there).
#include <hip/hip_runtime.h>

#define RT_MINREG_TU
#include "rt_internal.h"
#include "trace_kernels.h"

namespace rt {
namespace dv {
#if RT_SPLIT_TU
// the Perlin tables (c_perm / c_grad3) are per translation unit and only trace.hip uploads its
// copy: a variant instantiated here must not reach the noise textures
static_assert((0u & FT_TEX) == 0 && (F_C5 & FT_TEX) == 0, "textured variants belong in trace.hip");
template __global__ void render_kernel<false, 0u>(SceneD, ParamsD, float*, int32_t*, unsigned long long*);
template __global__ void render_kernel<false, F_C5>(SceneD, ParamsD, float*, int32_t*, unsigned long long*);
#endif
}  // namespace dv
}  // namespace rt
