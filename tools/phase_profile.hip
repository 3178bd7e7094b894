// Diagnostic build: per-phase cycle shares of the IPM kernel (s_memtime stamps).
// Not a timing build — read the shares, not the absolute time.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DMCPX_STAMPS=1 \
//          tools/phase_profile.hip mcp_amd/csrc/mcpx_api.cpp -o tools/phase_profile
// Run:   tools/phase_profile n m B {spec|gen|gen64|dense|schur|schurgen}
#include "../mcp_amd/csrc/ipm_kernel_impl.hpp"

#include <cstdio>
#include <cstring>
#include <cmath>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 32, m = argc > 2 ? atoi(argv[2]) : 16;
  const int B = argc > 3 ? atoi(argv[3]) : 16384;
  const int p = n * n + m * n + m + n;
  std::mt19937_64 g(7);
  std::normal_distribution<double> nd;
  std::vector<double> th((size_t)B * p);
  for (int b = 0; b < B; ++b) {
    double* t = &th[(size_t)b * p];
    std::vector<double> P(n * n);
    for (auto& v : P) v = nd(g);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double acc = 0;
        for (int k = 0; k < n; ++k) acc += P[k * n + i] * P[k * n + j];
        t[j * n + i] = acc;
      }
    for (int i = n * n; i < p; ++i) t[i] = nd(g);
  }
  mcpx_desc d{0, n, m, 0, B, p};
  mcpx_params prm;
  prm.max_inner_iters = 20;
  prm.max_outer_iters = 50;
  prm.tol = 1e-6;
  double *dth, *x, *y, *s, *kkt, *eps;
  int *outer, *status, *newton;
  uint64_t* stamps;
  (void)hipMalloc(&dth, th.size() * 8);
  (void)hipMemcpy(dth, th.data(), th.size() * 8, hipMemcpyHostToDevice);
  (void)hipMalloc(&x, (size_t)B * n * 8); (void)hipMalloc(&y, (size_t)B * m * 8); (void)hipMalloc(&s, (size_t)B * m * 8);
  (void)hipMalloc(&kkt, B * 8); (void)hipMalloc(&eps, B * 8);
  (void)hipMalloc(&outer, B * 4); (void)hipMalloc(&status, B * 4); (void)hipMalloc(&newton, B * 4);
  (void)hipMalloc(&stamps, (size_t)B * MCPX_NSTAMP * 8);
  mcpx::KernelArgs a;
  // reuse the ABI's parameter preparation through a normal call first (fills nothing here)
  std::memset((void*)&a, 0, sizeof a);
  a.theta = dth; a.theta_ld = p; a.x = x; a.y = y; a.s = s; a.kkt_error = kkt; a.eps = eps;
  a.outer_iters = outer; a.status = status; a.newton_iters = newton; a.stamps = stamps;
  a.n = n; a.m = m; a.max_inner = prm.max_inner_iters; a.max_outer = prm.max_outer_iters; a.tol = prm.tol;
  a.decay = 0.5; a.c_tau = 1.0 - 0.995; a.n_trials = 15;
  for (int k = 0; k <= prm.max_inner_iters; ++k) { a.tight[k] = 1 - exp(-0.1 * k); a.loose[k] = 1 + exp(-0.5 * k); }
  const char* mode = argc > 4 ? argv[4] : "spec";
  a.family = 0;
  a.solver = !strcmp(mode, "dense") ? MCPX_LINSOLVE_DENSE
             : (!strncmp(mode, "schur", 5) ? MCPX_LINSOLVE_SCHUR : MCPX_LINSOLVE_REDUCED);
  for (int rep = 0; rep < 2; ++rep) {
    hipError_t e = hipErrorInvalidValue;
    if (!strcmp(mode, "spec") && n == 32 && m == 16) e = mcpx::launch_one<48, 0, 32, 16, MCPX_LINSOLVE_REDUCED>(a, B, 0);
    else if (!strcmp(mode, "spec") && n == 16 && m == 8) e = mcpx::launch_one<24, 0, 16, 8, MCPX_LINSOLVE_REDUCED>(a, B, 0);
    else if (!strcmp(mode, "gen") && n + m <= 48) e = mcpx::launch_one<48, 0, 0, 0, MCPX_LINSOLVE_REDUCED>(a, B, 0);
    else if (!strcmp(mode, "gen64")) e = mcpx::launch_one<64, 0, 0, 0, MCPX_LINSOLVE_REDUCED>(a, B, 0);
    else if (!strcmp(mode, "dense")) e = mcpx::launch_one<64, 0, 0, 0, MCPX_LINSOLVE_DENSE>(a, B, 0);
    else if (!strcmp(mode, "schur") && n == 32 && m == 16) e = mcpx::launch_one<32, 0, 32, 16, MCPX_LINSOLVE_SCHUR>(a, B, 0);
    else if (!strcmp(mode, "schur") && n == 16 && m == 8) e = mcpx::launch_one<16, 0, 16, 8, MCPX_LINSOLVE_SCHUR>(a, B, 0);
    else if (!strcmp(mode, "schurgen") && n <= 32) e = mcpx::launch_one<32, 0, 0, 0, MCPX_LINSOLVE_SCHUR>(a, B, 0);
    if (e != hipSuccess) { printf("launch failed / unsupported mode: %s\n", hipGetErrorString(e)); return 1; }
    (void)hipDeviceSynchronize();
  }
  std::vector<uint64_t> st((size_t)B * MCPX_NSTAMP);
  std::vector<int> nw(B);
  (void)hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(nw.data(), newton, B * 4, hipMemcpyDeviceToHost);
  double tot[MCPX_NSTAMP] = {}, nsteps = 0, all = 0;
  for (int b = 0; b < B; ++b) { for (int i = 0; i < MCPX_NSTAMP; ++i) tot[i] += st[(size_t)b * MCPX_NSTAMP + i]; nsteps += nw[b]; }
  for (int i = 0; i < MCPX_NSTAMP; ++i) all += tot[i];
  const char* nm[] = {"residuals", "kkt-norm+rr", "schur-form", "LU/GJ", "backsub", "linesearch+update"};
  printf("[%s] n=%d m=%d B=%d  mean newton %.2f  wave-cycles per Newton step %.0f\n", mode, n, m, B, nsteps / B, all / nsteps);
  for (int i = 0; i < MCPX_NSTAMP; ++i) printf("  %-18s %5.1f%%  %8.0f cyc/step\n", nm[i], 100 * tot[i] / all, tot[i] / nsteps);
  return 0;
}
