// Runtime-(n, m) instantiations: affine family with ∂H/∂y ≡ 0, MFMA Schur-complement
// Newton solve (ipm_solve_kernel, AFF: R in A's place, −Qᵀ / −h / −g in LDS).
#include "ipm_kernel_impl.hpp"

namespace mcpx {

hipError_t launch_ipm_schur_aff(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st) {
  switch (nmax) {
    case 8: return launch_one<8, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    case 16: return launch_one<16, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    case 24: return launch_one<24, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    case 32: return launch_one<32, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    case 48: return launch_one<48, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    case 64: return launch_one<64, 1, 0, 0, MCPX_LINSOLVE_SCHUR>(a, batch, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mcpx
