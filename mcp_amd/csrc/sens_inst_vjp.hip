// vjp_kernel instantiations (sens_kernel_impl.hpp) for NMAX ∈ {8,16,24,32,48,64} ≥ n + m,
// QP and affine families.  One translation unit so the build compiles it in parallel.
#include "sens_kernel_impl.hpp"

namespace mcpx {

namespace {
template <int NMAX>
hipError_t go_vjp(const SensArgs& a, int64_t batch, hipStream_t st) {
  if (a.family == MCPX_FAMILY_QP)
    hipLaunchKernelGGL((vjp_kernel<NMAX, 0>), dim3((unsigned)batch), dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL((vjp_kernel<NMAX, 1>), dim3((unsigned)batch), dim3(64), 0, st, a);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_vjp(int nmax, const SensArgs& a, int64_t batch, hipStream_t st) {
  switch (nmax) {
    case 8: return go_vjp<8>(a, batch, st);
    case 16: return go_vjp<16>(a, batch, st);
    case 24: return go_vjp<24>(a, batch, st);
    case 32: return go_vjp<32>(a, batch, st);
    case 48: return go_vjp<48>(a, batch, st);
    case 64: return go_vjp<64>(a, batch, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mcpx
