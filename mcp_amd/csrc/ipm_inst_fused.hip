// The SCHUR QP solve with the rrule pullback fused into its epilogue
// (mcpx_solve_vjp_batch_device; BASELINE C5): compile-time (n, m) of the README QP,
// C2 and C3/C5, VJP register width = the smallest one-wave width ≥ n + m.
#include "sens_kernel_impl.hpp"

namespace mcpx {

bool has_fused_vjp(int family, int solver, int n, int m) {
  return family == MCPX_FAMILY_QP && solver == MCPX_LINSOLVE_SCHUR &&
         ((n == 2 && m == 2) || (n == 16 && m == 8) || (n == 32 && m == 16));
}

hipError_t launch_ipm_fused_vjp(int family, int solver, int n, int m, const KernelArgs& a, int64_t batch,
                                hipStream_t st) {
  if (family != MCPX_FAMILY_QP || solver != MCPX_LINSOLVE_SCHUR) return hipErrorNotFound;
  if (n == 2 && m == 2) return launch_one<2, 0, 2, 2, MCPX_LINSOLVE_SCHUR, 8>(a, batch, st);
  if (n == 16 && m == 8) return launch_one<16, 0, 16, 8, MCPX_LINSOLVE_SCHUR, 24>(a, batch, st);
  if (n == 32 && m == 16) return launch_one<32, 0, 32, 16, MCPX_LINSOLVE_SCHUR, 48>(a, batch, st);
  return hipErrorNotFound;
}

}  // namespace mcpx
