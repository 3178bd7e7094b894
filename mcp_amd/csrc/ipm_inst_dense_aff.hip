// Runtime-(n, m) instantiations: family AFFINE, full (n+2m)-dim Newton system.
#include "ipm_kernel_impl.hpp"

namespace mcpx {

hipError_t launch_ipm_dense_aff(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st) {
  switch (nmax) {
    case 8: return launch_one<8, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 16: return launch_one<16, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 24: return launch_one<24, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 32: return launch_one<32, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 48: return launch_one<48, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 64: return launch_one<64, 1, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mcpx
