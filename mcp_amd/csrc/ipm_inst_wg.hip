// Workgroup-per-instance kernels of the QP and affine families (ipm_wg_impl.hpp):
// MCPX_LINSOLVE_REDUCED / _DENSE at vector dimension buckets 128 … 768.
#include "ipm_wg_impl.hpp"

namespace mcpx {

template <int FAMILY, int SOLVER, int NV>
__global__ __launch_bounds__(wg::kThreads) void ipm_wg_kernel_t(const wg::WgArgs args) {
  wg::solve_instances<FAMILY, SOLVER, NV, NV, wg::NoGen>(args);
}

namespace {
template <int FAMILY, int SOLVER>
const void* pick(int nv) {
  switch (nv) {
    case 128: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 128>;
    case 256: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 256>;
    case 512: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 512>;
    case 768: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 768>;
    default: return nullptr;
  }
}
}  // namespace

const void* ipm_wg_kernel(int family, int solver, int nv) {
  const bool qp = family == MCPX_FAMILY_QP;
  if (family != MCPX_FAMILY_QP && family != MCPX_FAMILY_AFFINE) return nullptr;
  switch (solver) {
    case MCPX_LINSOLVE_REDUCED:
      return qp ? pick<MCPX_FAMILY_QP, MCPX_LINSOLVE_REDUCED>(nv) : pick<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_REDUCED>(nv);
    case MCPX_LINSOLVE_DENSE:
      return qp ? pick<MCPX_FAMILY_QP, MCPX_LINSOLVE_DENSE>(nv) : pick<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_DENSE>(nv);
    default:
      return nullptr;
  }
}

hipError_t launch_ipm_wg(int family, int solver, int nv, const wg::WgArgs& a, int grid, hipStream_t st) {
  const void* k = ipm_wg_kernel(family, solver, nv);
  if (!k) return hipErrorInvalidValue;
  void* params[] = {(void*)&a};
  return hipLaunchKernel(k, dim3((unsigned)grid), dim3(wg::kThreads), params, 0, st);
}

}  // namespace mcpx
