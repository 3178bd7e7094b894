// Diagnostic: per-phase s_memtime cycles of a generated nonlinear module's one-wave kernel
// (module built with -DMCPX_STAMPS=1; see tools/nl_phase.py, which writes θ and runs this).
//   nl_phase <module.hsaco> <kernel> <theta.bin> n m p B [threads per instance: 64, or 256 for _mw]
// A kernel name ending in "_wg" runs the workgroup-per-instance kernel the way the C ABI does
// (csrc/mcpx_api.cpp launch_wg: resident grid, atomic work queue, per-slot workspace).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../mcp_amd/csrc/ipm_kernel.h"
#include "../mcp_amd/csrc/ipm_wg.h"

int main(int argc, char** argv) {
  if (argc < 8) { fprintf(stderr, "usage\n"); return 2; }
  const char *mod = argv[1], *kname = argv[2], *thf = argv[3];
  const int n = atoi(argv[4]), m = atoi(argv[5]), p = atoi(argv[6]), B = atoi(argv[7]);
  const unsigned threads = argc > 8 ? (unsigned)atoi(argv[8]) : 64u;
  const int NST = argc > 9 ? atoi(argv[9]) : 4;  // stamps per instance (5: the LU elimination split out)
  std::vector<double> th((size_t)B * p);
  FILE* f = fopen(thf, "rb");
  if (!f || fread(th.data(), 8, th.size(), f) != th.size()) { fprintf(stderr, "theta read failed\n"); return 2; }
  fclose(f);
  hipModule_t M;
  hipFunction_t K;
  if (hipModuleLoad(&M, mod) != hipSuccess || hipModuleGetFunction(&K, M, kname) != hipSuccess) {
    fprintf(stderr, "module/kernel load failed\n");
    return 2;
  }
  double *dth, *x, *y, *s, *kkt, *eps;
  int *outer, *status, *newton;
  uint64_t* stamps;
  (void)hipMalloc(&dth, th.size() * 8);
  (void)hipMemcpy(dth, th.data(), th.size() * 8, hipMemcpyHostToDevice);
  (void)hipMalloc(&x, (size_t)B * n * 8); (void)hipMalloc(&y, (size_t)B * m * 8); (void)hipMalloc(&s, (size_t)B * m * 8);
  (void)hipMalloc(&kkt, B * 8); (void)hipMalloc(&eps, B * 8);
  (void)hipMalloc(&outer, B * 4); (void)hipMalloc(&status, B * 4); (void)hipMalloc(&newton, B * 4);
  (void)hipMalloc(&stamps, (size_t)B * NST * 8);
  mcpx::KernelArgs a{};
  a.theta = dth; a.theta_ld = p; a.x = x; a.y = y; a.s = s; a.kkt_error = kkt; a.eps = eps;
  a.outer_iters = outer; a.status = status; a.newton_iters = newton; a.stamps = stamps;
  a.n = n; a.m = m; a.family = MCPX_FAMILY_NONLINEAR; a.solver = MCPX_LINSOLVE_SCHUR;
  a.max_inner = 20; a.max_outer = 50; a.n_trials = 15; a.tol = 1e-6; a.decay = 0.5; a.c_tau = 1.0 - 0.995;
  for (int k = 0; k <= a.max_inner; ++k) { a.tight[k] = 1 - exp(-0.1 * k); a.loose[k] = 1 + exp(-0.5 * k); }
  size_t sz = sizeof a;
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  const size_t kl = strlen(kname);
  const bool wg = kl > 3 && !strcmp(kname + kl - 3, "_wg");
  mcpx::wg::WgArgs w{};
  size_t wsz = sizeof w;
  void* wcfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &w, HIP_LAUNCH_PARAM_BUFFER_SIZE, &wsz, HIP_LAUNCH_PARAM_END};
  unsigned grid = (unsigned)B;
  if (wg) {  // as launch_wg: SCHUR, ns = n
    int32_t meta[12] = {};
    hipDeviceptr_t mp;
    size_t mb = 0;
    if (hipModuleGetGlobal(&mp, &mb, M, "mcpx_nl_meta") != hipSuccess) { fprintf(stderr, "no mcpx_nl_meta\n"); return 2; }
    (void)hipMemcpy(meta, (void*)mp, std::min(mb, sizeof meta), hipMemcpyDeviceToHost);
    int per_cu = 0, cus = 0;
    (void)hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K, threads, 0);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto align = [](int64_t v) { return (v + 31) / 32 * 32; };
    const int ns = n;
    w.ld = ns + 1;
    w.off_blk = align((int64_t)ns * w.ld);
    w.off_aux = align(w.off_blk + meta[6]);
    w.off_rd = w.off_aux;
    w.slot_stride = align(w.off_aux + 4 * (int64_t)m);
    grid = (unsigned)std::min<int64_t>((int64_t)std::max(per_cu, 1) * std::max(cus, 1), B);
    double* ws = nullptr;
    (void)hipMalloc(&ws, sizeof(double) * (size_t)(grid * w.slot_stride) + 256);
    w.work = ws;
    w.counter = (int32_t*)(ws + grid * w.slot_stride);
    w.batch = B;
    w.k = a;
    printf("workgroup kernel: %d per CU, grid %u, slot %lld doubles\n", per_cu, grid, (long long)w.slot_stride);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(e0, 0);
    if (wg) (void)hipMemset(w.counter, 0, 4);
    if (hipModuleLaunchKernel(K, grid, 1, 1, threads, 1, 1, 0, 0, nullptr, wg ? wcfg : cfg) != hipSuccess) { fprintf(stderr, "launch failed\n"); return 2; }
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  std::vector<uint64_t> st((size_t)B * NST);
  std::vector<int> nw(B), stt(B);
  (void)hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(nw.data(), newton, B * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(stt.data(), status, B * 4, hipMemcpyDeviceToHost);
  const char* nm[] = {"eval+F+kkt", "schur prep+form", "LU (rest)", "dy/ds+linesearch+update", "LU elimination (2-D)", "2-D LU rejected (count)"};
  if (NST == 8) {  // the workgroup kernel's diagnostic build: four phases, then the LU's parts
    const char* nm8[] = {"eval+F+kkt", "schur prep+entries", "LU (all)", "dy/ds+linesearch+update",
                         "  LU: entries into tiles", "  LU: panel factor", "  LU: panel back + U12", "  LU: trailing (MFMA)"};
    for (int grp = 0; grp < 2; ++grp) {
      double tot[8] = {}, steps = 0;
      int cnt = 0;
      for (int b = 0; b < B; ++b) {
        if ((stt[b] != 0) != (grp == 1)) continue;
        for (int i = 0; i < 8; ++i) tot[i] += st[(size_t)b * 8 + i];
        steps += nw[b];
        ++cnt;
      }
      printf("[%s] %s: %d instances, %.0f Newton steps\n", kname, grp ? "failed" : "solved", cnt, steps);
      for (int i = 0; i < 8; ++i) printf("  %-28s %10.0f cyc/step\n", nm8[i], steps ? tot[i] / steps : 0.0);
    }
    return 0;
  }
  for (int grp = 0; grp < 2; ++grp) {  // solved, failed
    double tot[8] = {0, 0, 0, 0, 0, 0, 0, 0}, steps = 0; int cnt = 0, mx = 0;
    for (int b = 0; b < B; ++b) {
      if ((stt[b] != 0) != (grp == 1)) continue;
      for (int i = 0; i < NST; ++i) tot[i] += st[(size_t)b * NST + i];
      steps += nw[b]; ++cnt; mx = nw[b] > mx ? nw[b] : mx;
    }
    const double all = tot[0] + tot[1] + tot[2] + tot[3] + (NST > 4 ? tot[4] : 0.0);
    printf("[%s] B=%d kernel %.3f ms  %s: %d instances, newton mean %.1f max %d, cycles per Newton step %.0f\n", kname,
           B, ms, grp ? "failed" : "solved", cnt, cnt ? steps / cnt : 0.0, mx, steps ? all / steps : 0.0);
    for (int i = 0; i < (NST > 5 ? 5 : NST); ++i) printf("  %-26s %5.1f%%  %8.0f cyc/step\n", nm[i], all ? 100 * tot[i] / all : 0.0, steps ? tot[i] / steps : 0.0);
    if (NST > 5) printf("  guessed 2-D LU rejected on %.2f %% of the steps\n", steps ? 100.0 * tot[5] / steps : 0.0);
    if (NST > 7) printf("  of LU (rest): 2-D back substitution %.0f, searched-LU fallback %.0f cyc/step\n",
                        steps ? tot[6] / steps : 0.0, steps ? tot[7] / steps : 0.0);
  }
  return 0;
}
