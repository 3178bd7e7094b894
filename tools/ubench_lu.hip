// LU microbenchmark on the lane-change Schur complements (tests/ab/ubench_lu_data.py dumps them):
// one 64-lane wave per instance (row per lane, NMAX = 40), cycles per factorisation +
// solve (s_memtime) of LU variants, and their solutions (bitwise checked on the host).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1
//        -I mcp_amd/csrc tools/ubench_lu.hip -o tools/ubench_data/ubench_lu
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ipm_kernel_impl.hpp"

using namespace mcpx;
constexpr int NM = 40;

#include <utility>
#include "../tools/ubench_lu_variants.inc"

template <int V>
__global__ __launch_bounds__(64) void lu_bench(const double* S, const uint64_t* pat, int B, int reps, double* X,
                                               unsigned long long* cyc, int* pks) {
  const int ln = threadIdx.x;
  const int b = blockIdx.x % B;
  const int i = ln < NM ? ln : 0;
  const double* row = S + ((size_t)b * NM + i) * (NM + 1);
  double a0[NM];
#pragma unroll
  for (int j = 0; j < NM; ++j) a0[j] = row[j];
  const double r0 = row[NM];
  const uint64_t sp = ln < NM ? pat[i] : 0ull;
  const double* Sb = S + (size_t)b * NM * (NM + 1);
  int pk = pks[(size_t)b * 64 + ln];  // guessed pivot sequence (from variant 0's run)
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    double a[NM];
#pragma unroll
    for (int j = 0; j < NM; ++j) a[j] = __builtin_amdgcn_readfirstlane(0) + a0[j];  // fresh copy each rep
    double dz = 0.0;
    int pkr = pk;
    bool ok = run_variant<V>(a, r0, NM, ln, dz, pkr, sp, Sb);
    acc += ok ? dz : 1e300;
    if (r == 0 && V == 0) pks[(size_t)b * 64 + ln] = pkr;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  X[(size_t)blockIdx.x * 64 + ln] = acc / reps;
  if (ln == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
}

int main(int argc, char** argv) {
  const int B = 256, reps = argc > 1 ? atoi(argv[1]) : 20;
  std::vector<double> S((size_t)B * NM * (NM + 1));
  std::vector<uint64_t> pat(NM);
  FILE* f = fopen("tools/ubench_data/lu_S.bin", "rb");
  fread(S.data(), sizeof(double), S.size(), f);
  fclose(f);
  f = fopen("tools/ubench_data/lu_pat.bin", "rb");
  fread(pat.data(), 8, NM, f);
  fclose(f);
  double *dS, *dX;
  uint64_t* dP;
  unsigned long long* dC;
  int* dpk;
  hipMalloc(&dS, S.size() * 8);
  hipMalloc(&dP, NM * 8);
  hipMalloc(&dX, (size_t)B * 64 * 8);
  hipMalloc(&dC, B * 8);
  hipMalloc(&dpk, (size_t)B * 64 * 4);
  hipMemset(dpk, 0, (size_t)B * 64 * 4);
  hipMemcpy(dS, S.data(), S.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dP, pat.data(), NM * 8, hipMemcpyHostToDevice);
  std::vector<double> X0((size_t)B * 64), X1((size_t)B * 64), X((size_t)B * 64);
  std::vector<unsigned long long> C(B);
#define RUN(V)                                                                                       \
  {                                                                                                  \
    hipLaunchKernelGGL(lu_bench<V>, dim3(B), dim3(64), 0, 0, dS, dP, B, reps, dX, dC, dpk);          \
    hipDeviceSynchronize();                                                                          \
    hipMemcpy(X.data(), dX, X.size() * 8, hipMemcpyDeviceToHost);                                    \
    hipMemcpy(C.data(), dC, B * 8, hipMemcpyDeviceToHost);                                           \
    if (V == 1) X1 = X;                                                                              \
    if (V == 4) X0 = X;                                                                              \
    double s = 0;                                                                                    \
    for (auto c : C) s += c;                                                                         \
    size_t diff = 0;                                                                                 \
    for (size_t q = 0; q < X.size(); ++q) diff += (X[q] != X0[q]) && !(X[q] != X[q] && X0[q] != X0[q]); \
    size_t diff1 = 0;                                                                                \
    for (size_t q = 0; q < X.size(); ++q) diff1 += (X[q] != X1[q]) && !(X[q] != X[q] && X1[q] != X1[q]); \
    printf("variant %d (%s): %8.0f cycles per LU+solve (mean of %d waves), entries differing from v4: %zu, from v1: %zu\n", \
           V, variant_name(V), s / B, B, diff, diff1);                                               \
  }
  RUN(0) RUN(1) RUN(4) RUN(9) RUN(11) RUN(12)
  return 0;
}
