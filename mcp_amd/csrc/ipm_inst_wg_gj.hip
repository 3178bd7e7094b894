// The QP family's workgroup SCHUR kernels (ipm_wg_impl.hpp with gj_vr.hpp): n ≤ 128 (beyond
// the one-wave SCHUR kernel's n + m ≤ 64), the Schur complement formed on the matrix cores and
// solved by the blocked Gauss-Jordan with MFMA trailing updates (pivoting LU when M is not
// symmetric or a pivot is not positive), at vector dimension n + 2m ≤ nv ∈ wg::kDimBuckets.
// A unit of its own: it builds in parallel with the other workgroup units.
#include "ipm_wg_impl.hpp"

namespace mcpx {

template <int NV>
__global__ __launch_bounds__(wg::kThreads) void ipm_wg_gj_kernel_t(const wg::WgArgs args) {
  wg::solve_instances<MCPX_FAMILY_QP, MCPX_LINSOLVE_SCHUR, NV, wg::kGjMax, wg::NoGen>(args);
}

const void* ipm_wg_gj_kernel(int nv) {
  switch (nv) {
    case 128: return (const void*)&ipm_wg_gj_kernel_t<128>;
    case 256: return (const void*)&ipm_wg_gj_kernel_t<256>;
    case 512: return (const void*)&ipm_wg_gj_kernel_t<512>;
    case 768: return (const void*)&ipm_wg_gj_kernel_t<768>;
    default: return nullptr;
  }
}

}  // namespace mcpx
