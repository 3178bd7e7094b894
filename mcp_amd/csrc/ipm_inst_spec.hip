// Compile-time-(n, m) instantiations of the slack-eliminated (RED) kernel for
// the BASELINE configurations: README QP (n = m = 2), C2 (16, 8), C3 (32, 16).
#include "ipm_kernel_impl.hpp"

namespace mcpx {

hipError_t launch_ipm_spec(int family, bool reduced, int n, int m, const KernelArgs& a, int64_t batch,
                           hipStream_t st) {
  if (family == MCPX_FAMILY_QP && reduced) {
    if (n == 2 && m == 2) return launch_one<4, 0, 2, 2, true>(a, batch, st);
    if (n == 16 && m == 8) return launch_one<24, 0, 16, 8, true>(a, batch, st);
    if (n == 32 && m == 16) return launch_one<48, 0, 32, 16, true>(a, batch, st);
  }
  return hipErrorNotFound;
}

}  // namespace mcpx
