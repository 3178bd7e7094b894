// Workgroup-per-instance sensitivity kernels of the QP and affine families
// (sens_wg_impl.hpp) for n + 2m beyond the one-wave kernels' 64 rows, at the vector
// dimension buckets 128 … 768 of the workgroup solver.
#include "sens_wg_impl.hpp"

namespace mcpx {

template <int FAMILY, bool JVP, int NV>
__global__ __launch_bounds__(wg::kThreads) void sens_wg_kernel_t(const wg::WgSensArgs args) {
  wg::sens_instances<FAMILY, JVP, NV, NV, wg::NoGen>(args);
}

namespace {
template <int FAMILY, bool JVP>
const void* pick(int nv) {
  switch (nv) {
    case 128: return (const void*)&sens_wg_kernel_t<FAMILY, JVP, 128>;
    case 256: return (const void*)&sens_wg_kernel_t<FAMILY, JVP, 256>;
    case 512: return (const void*)&sens_wg_kernel_t<FAMILY, JVP, 512>;
    case 768: return (const void*)&sens_wg_kernel_t<FAMILY, JVP, 768>;
    default: return nullptr;
  }
}
}  // namespace

const void* sens_wg_kernel(int family, bool jvp, int nv) {
  if (family == MCPX_FAMILY_QP) return jvp ? pick<MCPX_FAMILY_QP, true>(nv) : pick<MCPX_FAMILY_QP, false>(nv);
  if (family == MCPX_FAMILY_AFFINE)
    return jvp ? pick<MCPX_FAMILY_AFFINE, true>(nv) : pick<MCPX_FAMILY_AFFINE, false>(nv);
  return nullptr;
}

hipError_t launch_sens_wg(int family, bool jvp, int nv, const wg::WgSensArgs& a, int grid, hipStream_t st) {
  const void* k = sens_wg_kernel(family, jvp, nv);
  if (!k) return hipErrorInvalidValue;
  void* params[] = {(void*)&a};
  return hipLaunchKernel(k, dim3((unsigned)grid), dim3(wg::kThreads), params, 0, st);
}

}  // namespace mcpx
