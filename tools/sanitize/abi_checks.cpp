// Host-side sanitizer driver (SURVEY.md §5 "Race detection / sanitizers"): the C
// ABI's host code (mcpx_api.cpp, compiled with -fsanitize=address,undefined on
// the host side only) exercised through every argument-checking and no-device
// path, from several threads at once (the thread-local error string, the
// reentrancy claim of include/mcpx.h).  Built and run by tools/sanitize/run.sh;
// needs no GPU (without one every compute call must return MCPX_ENODEV).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/mcpx.h"

static int failures = 0;
#define EXPECT(cond)                                                  \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static void one_thread(int seed) {
  const bool gpu = mcpx_device_count() > 0;
  mcpx_params p;
  std::memset(&p, 0xAB, sizeof p);  // garbage first: mcpx_default_params must set every field
  mcpx_default_params(&p);
  EXPECT(p.tol == 1e-4 && p.max_inner_iters == 20 && p.max_outer_iters == 50 && p.kernel == MCPX_KERNEL_AUTO);
  EXPECT(p.linear_solver == MCPX_LINSOLVE_REDUCED);
  const int n = 3 + seed % 5, m = 2 + seed % 3;
  const int64_t pdim = mcpx_theta_dim(MCPX_FAMILY_QP, n, m);
  EXPECT(pdim == (int64_t)n * n + m * n + m + n);
  EXPECT(mcpx_theta_dim(7, n, m) < 0 && mcpx_theta_dim(MCPX_FAMILY_QP, -1, m) < 0);
  const int B = 4;
  std::vector<double> theta(B * pdim, 0.5), x(B * n), y(B * m), s(B * m), kkt(B), eps(B);
  std::vector<int32_t> outer(B), status(B), newton(B);
  mcpx_out o{};
  o.x = x.data(); o.y = y.data(); o.s = s.data(); o.kkt_error = kkt.data(); o.eps = eps.data();
  o.outer_iters = outer.data(); o.status = status.data(); o.newton_iters = newton.data();
  mcpx_desc d{MCPX_FAMILY_QP, n, m, 0, B, pdim};
  // argument errors: never touch the buffers, always leave a message
  mcpx_desc bad = d;
  bad.theta_ld = pdim - 1;
  EXPECT(mcpx_solve_batch(&bad, theta.data(), nullptr, nullptr, nullptr, &p, 1, &o) == MCPX_EINVAL);
  EXPECT(std::strlen(mcpx_last_error()) > 0);
  bad = d;
  bad.batch = -1;
  EXPECT(mcpx_solve_batch(&bad, theta.data(), nullptr, nullptr, nullptr, &p, 1, &o) == MCPX_EINVAL);
  EXPECT(mcpx_solve_batch(nullptr, theta.data(), nullptr, nullptr, nullptr, &p, 1, &o) == MCPX_EINVAL);
  EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, nullptr, 1, &o) == MCPX_EINVAL);
  mcpx_params q = p;
  q.kernel = 9;
  EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, &q, 1, &o) == MCPX_EINVAL);
  q = p;
  q.decay = std::nan("");
  EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, &q, 1, &o) == MCPX_EINVAL);
  q = p;
  q.max_inner_iters = 100000;
  EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, &q, 1, &o) == MCPX_EUNSUPPORTED);
  q = p;
  q.linear_solver = MCPX_LINSOLVE_SCHUR;
  mcpx_desc big{MCPX_FAMILY_QP, 130, 20, 0, 1, mcpx_theta_dim(MCPX_FAMILY_QP, 130, 20)};  // QP SCHUR: n ≤ 128
  EXPECT(mcpx_solve_batch(&big, theta.data(), nullptr, nullptr, nullptr, &q, 1, &o) == MCPX_EUNSUPPORTED);
  mcpx_out none{};
  EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, &p, 1, &none) == MCPX_EINVAL);
  // sensitivities: argument checks
  std::vector<double> dth(B * pdim);
  EXPECT(mcpx_vjp_batch(&d, nullptr, x.data(), y.data(), s.data(), nullptr, nullptr, nullptr, 1, dth.data(),
                        nullptr) == MCPX_EINVAL);
  EXPECT(mcpx_jvp_batch(&d, theta.data(), x.data(), y.data(), s.data(), -1, nullptr, 1, dth.data(), nullptr) ==
         MCPX_EINVAL);
  // module loading: missing / empty / foreign files
  mcpx_module* mod = nullptr;
  EXPECT(mcpx_module_load("/nonexistent/file.hsaco", &mod) == MCPX_EINVAL && mod == nullptr);
  EXPECT(mcpx_module_load(nullptr, &mod) == MCPX_EINVAL);
  EXPECT(mcpx_module_dims(nullptr, nullptr, nullptr, nullptr, nullptr) == MCPX_EINVAL);
  mcpx_module_unload(nullptr);
  if (!gpu) {  // a valid call without a device: an error, never a CPU fallback
    EXPECT(mcpx_solve_batch(&d, theta.data(), nullptr, nullptr, nullptr, &p, 1, &o) == MCPX_ENODEV);
    EXPECT(mcpx_vjp_batch(&d, theta.data(), x.data(), y.data(), s.data(), nullptr, nullptr, nullptr, 1,
                          dth.data(), nullptr) == MCPX_ENODEV);
  }
}

int main() {
  EXPECT(mcpx_version() == MCPX_VERSION);
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) ts.emplace_back(one_thread, t);
  for (auto& t : ts) t.join();
  std::printf("abi_checks: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
