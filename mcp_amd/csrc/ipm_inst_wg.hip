// Workgroup-per-instance kernels of the QP and affine families (ipm_wg_impl.hpp):
// MCPX_LINSOLVE_REDUCED / _DENSE at vector dimension buckets 128 … 768.  Bucket 128 and
// the systems of at most MCPX_VR_MAX rows in bucket 256 (REDUCED at KKT 256: n + m = 192)
// take the register-resident LU (lu_vr.hpp); those kernels are compiled in their own
// unit, ipm_inst_wg_vr.hip (they dominate the build), and reached through ipm_wg_vr_kernel.
#include "ipm_wg_impl.hpp"

namespace mcpx {

template <int FAMILY, int SOLVER, int NV, int NS = NV>
__global__ __launch_bounds__(wg::kThreads) void ipm_wg_kernel_t(const wg::WgArgs args) {
  wg::solve_instances<FAMILY, SOLVER, NV, NS, wg::NoGen>(args);
}

namespace {
template <int FAMILY, int SOLVER>
const void* pick(int nv, int ns) {
  if (nv == 128 || (nv == 256 && ns <= MCPX_VR_MAX)) return ipm_wg_vr_kernel(FAMILY, SOLVER, nv);
  switch (nv) {
    case 256: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 256>;
    case 512: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 512>;
    case 768: return (const void*)&ipm_wg_kernel_t<FAMILY, SOLVER, 768>;
    default: return nullptr;
  }
}
}  // namespace

const void* ipm_wg_kernel(int family, int solver, int nv, int ns) {
  const bool qp = family == MCPX_FAMILY_QP;
  if (family != MCPX_FAMILY_QP && family != MCPX_FAMILY_AFFINE) return nullptr;
  switch (solver) {
    case MCPX_LINSOLVE_REDUCED:
      return qp ? pick<MCPX_FAMILY_QP, MCPX_LINSOLVE_REDUCED>(nv, ns) : pick<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_REDUCED>(nv, ns);
    case MCPX_LINSOLVE_DENSE:
      return qp ? pick<MCPX_FAMILY_QP, MCPX_LINSOLVE_DENSE>(nv, ns) : pick<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_DENSE>(nv, ns);
    case MCPX_LINSOLVE_SCHUR:  // the QP family, n ≤ 128 (gj_vr.hpp)
      return qp && ns <= wg::kGjMax ? ipm_wg_gj_kernel(nv) : nullptr;
    default:
      return nullptr;
  }
}

hipError_t launch_ipm_wg(int family, int solver, int nv, int ns, const wg::WgArgs& a, int grid, hipStream_t st) {
  const void* k = ipm_wg_kernel(family, solver, nv, ns);
  if (!k) return hipErrorInvalidValue;
  void* params[] = {(void*)&a};
  return hipLaunchKernel(k, dim3((unsigned)grid), dim3(wg::kThreads), params, 0, st);
}

}  // namespace mcpx
