// Compile-time-(n, m) instantiations for the BASELINE configurations:
// README QP (n = m = 2), C2 (16, 8), C3 (32, 16), for the slack-eliminated
// (REDUCED) and the MFMA Schur-complement (SCHUR) Newton solves; C3's shape also
// for the affine family's SCHUR solve (∂H/∂y ≡ 0).
#include "ipm_kernel_impl.hpp"

namespace mcpx {

hipError_t launch_ipm_spec(int family, int solver, int n, int m, const KernelArgs& a, int64_t batch,
                           hipStream_t st) {
  if (family == MCPX_FAMILY_AFFINE && solver == MCPX_LINSOLVE_SCHUR) {  // C3's shape through the affine layout
    if (n == 32 && m == 16) return launch_one<32, 1, 32, 16, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    return hipErrorNotFound;
  }
  if (family != MCPX_FAMILY_QP) return hipErrorNotFound;
  if (solver == MCPX_LINSOLVE_REDUCED) {
    if (n == 2 && m == 2) return launch_one<4, 0, 2, 2, MCPX_LINSOLVE_REDUCED>(a, batch, st);
    if (n == 16 && m == 8) return launch_one<24, 0, 16, 8, MCPX_LINSOLVE_REDUCED>(a, batch, st);
    if (n == 32 && m == 16) return launch_one<48, 0, 32, 16, MCPX_LINSOLVE_REDUCED>(a, batch, st);
  }
  if (solver == MCPX_LINSOLVE_SCHUR) {
    if (n == 2 && m == 2) return launch_one<2, 0, 2, 2, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    if (n == 16 && m == 8) return launch_one<16, 0, 16, 8, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    if (n == 32 && m == 16) return launch_one<32, 0, 32, 16, MCPX_LINSOLVE_SCHUR>(a, batch, st);
  }
  return hipErrorNotFound;
}

}  // namespace mcpx
