// Register-resident workgroup kernels of the QP and affine families (ipm_wg_impl.hpp with
// lu_vr.hpp): MCPX_LINSOLVE_REDUCED / _DENSE in bucket 128 (every system ≤ 128 rows) and in
// bucket 256 for systems of at most MCPX_VR_MAX rows.  A unit of their own: their unrolled
// tile loops make them the slowest kernels to compile, and the other workgroup kernels
// (ipm_inst_wg.hip) build in parallel.
#include "ipm_wg_impl.hpp"

namespace mcpx {

template <int FAMILY, int SOLVER, int NV, int NS>
__global__ __launch_bounds__(wg::kThreads) void ipm_wg_vr_kernel_t(const wg::WgArgs args) {
  static_assert(wg::kVr<NS>, "a register-resident instance");
  wg::solve_instances<FAMILY, SOLVER, NV, NS, wg::NoGen>(args);
}

namespace {
template <int FAMILY, int SOLVER>
const void* pick_vr(int nv) {
  if (nv == 128) return (const void*)&ipm_wg_vr_kernel_t<FAMILY, SOLVER, 128, 128>;
  if (nv == 256) return (const void*)&ipm_wg_vr_kernel_t<FAMILY, SOLVER, 256, MCPX_VR_MAX>;
  return nullptr;
}
}  // namespace

const void* ipm_wg_vr_kernel(int family, int solver, int nv) {
  const bool qp = family == MCPX_FAMILY_QP;
  if (family != MCPX_FAMILY_QP && family != MCPX_FAMILY_AFFINE) return nullptr;
  switch (solver) {
    case MCPX_LINSOLVE_REDUCED:
      return qp ? pick_vr<MCPX_FAMILY_QP, MCPX_LINSOLVE_REDUCED>(nv) : pick_vr<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_REDUCED>(nv);
    case MCPX_LINSOLVE_DENSE:
      return qp ? pick_vr<MCPX_FAMILY_QP, MCPX_LINSOLVE_DENSE>(nv) : pick_vr<MCPX_FAMILY_AFFINE, MCPX_LINSOLVE_DENSE>(nv);
    default:
      return nullptr;
  }
}

}  // namespace mcpx
