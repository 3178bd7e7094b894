// Runtime-(n, m) instantiations: family QP, full (n+2m)-dim Newton system.
#include "ipm_kernel_impl.hpp"

namespace mcpx {

hipError_t launch_ipm_dense_qp(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st) {
  switch (nmax) {
    case 8: return launch_one<8, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 16: return launch_one<16, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 24: return launch_one<24, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 32: return launch_one<32, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 48: return launch_one<48, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    case 64: return launch_one<64, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, batch, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mcpx
