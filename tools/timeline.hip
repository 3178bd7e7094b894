// Diagnostic build: the residency timeline of one SCHUR launch (MCPX_STAMPS=2).
// Every wave records its start and end on the 100 MHz constant clock (s_memrealtime) and
// the slot it ran in (HW_ID: wave / SIMD / CU / SE, XCC_ID); pass 1 and pass 2 are timed
// apart with HIP events.  tools/timeline.py writes θ (the bench's own inputs), runs this
// and reads the result.  Not a timing build of the product: the stamps add two stores.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DMCPX_STAMPS=2 \
//          tools/timeline.hip -o tools/timeline
// Run:   tools/timeline theta.bin out.bin [reps]
//   theta.bin: int32 n, m, B, then B·p fp64 (QP layout of include/mcpx.h)
//   out.bin:   fp64 pass-1 ms, pass-2 ms (median of reps), then per instance
//              uint64 start, end, hw_id, xcc_id, pass, and int32 newton, status
#include "../mcp_amd/csrc/ipm_kernel_impl.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <int NC, int MC, int P>
static void launch(const mcpx::KernelArgs& a, int B) {
  hipLaunchKernelGGL((mcpx::ipm_solve_kernel<NC, 0, NC, MC, MCPX_LINSOLVE_SCHUR, P, 0>), dim3((unsigned)B), dim3(64), 0,
                     0, a);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s theta.bin out.bin [reps]\n", argv[0]);
    return 2;
  }
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hdr[3];
  if (fread(hdr, 4, 3, f) != 3) return 2;
  const int n = hdr[0], m = hdr[1], B = hdr[2];
  const int p = n * n + m * n + m + n;
  if (!((n == 32 && m == 16) || (n == 16 && m == 8)) || B < 1) {
    fprintf(stderr, "timeline: only the C3 (32, 16) and C2 (16, 8) SCHUR kernels (got n=%d m=%d B=%d)\n", n, m, B);
    return 2;
  }
  std::vector<double> th((size_t)B * p);
  if (fread(th.data(), 8, th.size(), f) != th.size()) return 2;
  fclose(f);

  double *dth, *x, *y, *s, *kkt, *eps;
  int *outer, *status, *newton;
  uint64_t* stamps;
  CK(hipMalloc(&dth, th.size() * 8));
  CK(hipMemcpy(dth, th.data(), th.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&x, (size_t)B * n * 8));
  CK(hipMalloc(&y, (size_t)B * m * 8));
  CK(hipMalloc(&s, (size_t)B * m * 8));
  CK(hipMalloc(&kkt, (size_t)B * 8));
  CK(hipMalloc(&eps, (size_t)B * 8));
  CK(hipMalloc(&outer, (size_t)B * 4));
  CK(hipMalloc(&status, (size_t)B * 4));
  CK(hipMalloc(&newton, (size_t)B * 4));
  CK(hipMalloc(&stamps, (size_t)B * MCPX_NSTAMP * 8));
  CK(hipMemset(stamps, 0, (size_t)B * MCPX_NSTAMP * 8));

  mcpx::KernelArgs a;
  std::memset((void*)&a, 0, sizeof a);
  a.theta = dth; a.theta_ld = p; a.x = x; a.y = y; a.s = s; a.kkt_error = kkt; a.eps = eps;
  a.outer_iters = outer; a.status = status; a.newton_iters = newton; a.stamps = stamps;
  a.n = n; a.m = m; a.solver = MCPX_LINSOLVE_SCHUR; a.family = 0;
  a.max_inner = 20; a.max_outer = 50; a.tol = 1e-6;  // bench.py's C3/C2 (mcpx_default_params, tol 1e-6)
  a.decay = 0.5; a.c_tau = 1.0 - 0.995; a.n_trials = 15;
  for (int k = 0; k <= a.max_inner; ++k) { a.tight[k] = 1 - exp(-0.1 * k); a.loose[k] = 1 + exp(-0.5 * k); }

  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  std::vector<float> t1, t2;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipEventRecord(e0, 0));
    if (n == 32) launch<32, 16, 1>(a, B); else launch<16, 8, 1>(a, B);
    CK(hipEventRecord(e1, 0));
    if (n == 32) launch<32, 16, 2>(a, B); else launch<16, 8, 2>(a, B);
    CK(hipEventRecord(e2, 0));
    CK(hipGetLastError());
    CK(hipEventSynchronize(e2));
    float a1, a2;
    CK(hipEventElapsedTime(&a1, e0, e1));
    CK(hipEventElapsedTime(&a2, e1, e2));
    if (r > 0) { t1.push_back(a1); t2.push_back(a2); }  // the first launch warms up
  }
  std::sort(t1.begin(), t1.end());
  std::sort(t2.begin(), t2.end());
  std::vector<uint64_t> st((size_t)B * MCPX_NSTAMP);
  std::vector<int32_t> nw(B), stt(B);
  CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(nw.data(), newton, (size_t)B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(stt.data(), status, (size_t)B * 4, hipMemcpyDeviceToHost));
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  const double ms[2] = {t1[t1.size() / 2], t2[t2.size() / 2]};
  fwrite(ms, 8, 2, o);
  for (int b = 0; b < B; ++b) {
    fwrite(&st[(size_t)b * MCPX_NSTAMP], 8, 5, o);
    fwrite(&nw[b], 4, 1, o);
    fwrite(&stt[b], 4, 1, o);
  }
  fclose(o);
  printf("timeline n=%d m=%d B=%d: pass 1 %.4f ms, pass 2 %.4f ms (median of %d)\n", n, m, B, ms[0], ms[1], reps);
  return 0;
}
