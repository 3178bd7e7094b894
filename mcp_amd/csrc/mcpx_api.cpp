// mcpx_api.cpp — implementation of the C ABI declared in include/mcpx.h.
//
// Host side of the drop-in boundary for src/solver.jl:35-122: argument checks
// (the reference's own ArgumentError / @assert sites, src/AutoDiff.jl:19-23,
// src/mcp.jl:191), the per-call constant tables the reference computes inline
// (line-search step sizes src/solver.jl:127-138, ϵ-schedule factors
// src/solver.jl:111-113), device selection, batch sharding over GPUs and
// stream-ordered launches.  Reentrant: no global mutable state apart from the
// thread-local error string.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mcpx.h"
#include "ipm_kernel.h"
#include "ipm_wg.h"
#include "sens_kernel.h"

// A generated nonlinear module (MCPX_FAMILY_NONLINEAR, include/mcpx.h): the
// code object image, its metadata record and the per-device loaded modules.
struct mcpx_module {
  std::vector<char> image;
  int32_t meta[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // mcpx_nl_meta of csrc/ipm_nl_kernel.hpp
  std::mutex mu;
  std::map<int, hipModule_t> loaded;  // device → module, loaded on first use
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(MCPX_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));            \
  } while (0)

int check_device(int dev) {
  static std::atomic<uint64_t> verified{0};  // devices already found to be gfx950 (bit per ordinal < 64)
  if (dev >= 0 && dev < 64 && ((verified.load(std::memory_order_relaxed) >> dev) & 1)) return MCPX_OK;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(MCPX_ENODEV, "device %d is %s; this build targets gfx950 (MI355X) only", dev,
                prop.gcnArchName);
  if (dev >= 0 && dev < 64) verified.fetch_or(uint64_t(1) << dev, std::memory_order_relaxed);
  return MCPX_OK;
}

// The current device of a device-buffer call: MCPX_ENODEV when none is visible.
int current_device(int* dev) {
  const hipError_t e = hipGetDevice(dev);
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return fail(MCPX_ENODEV, "no HIP device visible");
  HIP_TRY(e);
  return check_device(*dev);
}

// MCPX_GENERIC_KERNELS=1 disables the compile-time-(n, m) kernels (A/B switch).
bool specialized_enabled() {
  const char* e = std::getenv("MCPX_GENERIC_KERNELS");
  return !(e && e[0] == '1');
}

// Register-row width of the runtime-(n, m) kernels: smallest compiled width ≥ N.
int pick_nmax(int N) {
  for (int w : {8, 16, 24, 32, 48, 64})
    if (N <= w) return w;
  return -1;
}

// Smallest workgroup-kernel vector-dimension bucket ≥ N (QP / affine), or -1.
int pick_wg_bucket(int N) {
  for (int w : mcpx::wg::kDimBuckets)
    if (N <= w) return w;
  return -1;
}

// Validates desc/params and fills the scalar part + tables of the kernel args.
// *wg: the solve runs on the workgroup-per-instance kernels (ipm_wg_impl.hpp);
// *nmax: the one-wave kernels' row width, or the workgroup kernels' dimension bucket.
int prepare(const mcpx_desc* d, const mcpx_params* p, mcpx::KernelArgs* a, int* nmax,
            const mcpx_module* mod = nullptr, bool* wg = nullptr, bool* mw = nullptr, bool* band = nullptr) {
  bool wg_local = false, mw_local = false, band_local = false;
  if (!wg) wg = &wg_local;
  if (!mw) mw = &mw_local;
  if (!band) band = &band_local;
  *mw = false;
  *band = false;
  if (!d || !p) return fail(MCPX_EINVAL, "desc and params must be non-NULL");
  int64_t pd;
  if (mod) {  // a generated nonlinear module: θ dimension and sizes from its metadata
    if (d->family != MCPX_FAMILY_NONLINEAR)
      return fail(MCPX_EINVAL, "a generated module solves family MCPX_FAMILY_NONLINEAR (got %d)", d->family);
    if (d->n != mod->meta[1] || d->m != mod->meta[2])
      return fail(MCPX_EINVAL, "desc (n=%d, m=%d) does not match the module (n=%d, m=%d)", d->n, d->m,
                  mod->meta[1], mod->meta[2]);
    pd = mod->meta[3];
  } else {
    if (d->family == MCPX_FAMILY_NONLINEAR)
      return fail(MCPX_EINVAL, "family MCPX_FAMILY_NONLINEAR runs through its generated module "
                  "(mcpx_solve_batch_module*)");
    pd = mcpx_theta_dim(d->family, d->n, d->m);
  }
  if (pd < 0) return fail(MCPX_EINVAL, "bad family %d or negative dimensions (n=%d, m=%d)", d->family, d->n, d->m);
  if (d->n + d->m < 1) return fail(MCPX_EINVAL, "empty problem (n = m = 0)");
  if (d->batch < 0) return fail(MCPX_EINVAL, "negative batch");
  if (d->theta_ld < pd) return fail(MCPX_EINVAL, "theta_ld %lld < parameter dimension %lld", (long long)d->theta_ld, (long long)pd);
  const int ls = p->linear_solver;
  if (ls != MCPX_LINSOLVE_REDUCED && ls != MCPX_LINSOLVE_DENSE && ls != MCPX_LINSOLVE_SCHUR)
    return fail(MCPX_EINVAL, "unknown linear_solver %d", ls);
  if (p->kernel != MCPX_KERNEL_AUTO && p->kernel != MCPX_KERNEL_WAVE && p->kernel != MCPX_KERNEL_WORKGROUP &&
      p->kernel != MCPX_KERNEL_MULTIWAVE && p->kernel != MCPX_KERNEL_BAND)
    return fail(MCPX_EINVAL, "unknown kernel selector %d", p->kernel);
  bool wave_ok, wg_ok;
  if (mod) {
    wave_ok = (mod->meta[5] >> ls) & 1;
    wg_ok = (mod->meta[5] >> (3 + ls)) & 1;
    const bool mw_ok = ls == MCPX_LINSOLVE_SCHUR && ((mod->meta[5] >> MCPX_MODULE_SCHUR_MW) & 1);
    if (p->kernel == MCPX_KERNEL_MULTIWAVE && !mw_ok)
      return fail(MCPX_EUNSUPPORTED, "the generated module has no multi-wave kernel for linear_solver=%d", ls);
    *mw = mw_ok && p->kernel == MCPX_KERNEL_MULTIWAVE;  // measured slower than one wave: opt-in
    // the band kernel (ipm_nl_band.hpp): forced, or AUTO when the module prefers it or has no
    // one-wave SCHUR kernel (oracle/ipm_oracle.c picks lu_band_solve by the same rule)
    const bool band_ok = ls == MCPX_LINSOLVE_SCHUR && ((mod->meta[5] >> MCPX_MODULE_BAND) & 1);
    const bool band_auto = band_ok && ((mod->meta[5] >> MCPX_MODULE_BAND_AUTO) & 1);
    if (p->kernel == MCPX_KERNEL_BAND && !band_ok)
      return fail(MCPX_EUNSUPPORTED, "the generated module has no band kernel for linear_solver=%d", ls);
    *band = p->kernel == MCPX_KERNEL_BAND || (p->kernel == MCPX_KERNEL_AUTO && band_ok && (band_auto || !wave_ok));
    *nmax = 0;
  } else {
    if (p->kernel == MCPX_KERNEL_MULTIWAVE)
      return fail(MCPX_EUNSUPPORTED, "MCPX_KERNEL_MULTIWAVE is a generated module's SCHUR kernel");
    if (p->kernel == MCPX_KERNEL_BAND)
      return fail(MCPX_EUNSUPPORTED, "MCPX_KERNEL_BAND is a generated module's SCHUR kernel");
    // (affine family: ∂H/∂y is taken as 0 — the S block of θ' is not read, include/mcpx.h)
    const int N = ls == MCPX_LINSOLVE_DENSE ? d->n + 2 * d->m : (ls == MCPX_LINSOLVE_REDUCED ? d->n + d->m : d->n);
    const int lanes = ls == MCPX_LINSOLVE_DENSE ? d->n + 2 * d->m : d->n + d->m;  // one wave: one lane per row
    wave_ok = pick_nmax(N) > 0 && lanes <= MCPX_MAX_KKT_DIM;
    // workgroup kernels: REDUCED / DENSE, and SCHUR for the QP family up to n = 128 (gj_vr.hpp)
    wg_ok = (ls != MCPX_LINSOLVE_SCHUR || (d->family == MCPX_FAMILY_QP && d->n <= mcpx::wg::kGjMax)) &&
            d->n + 2 * d->m <= MCPX_MAX_WG_KKT_DIM;
    *nmax = wave_ok && p->kernel != MCPX_KERNEL_WORKGROUP ? pick_nmax(N) : pick_wg_bucket(d->n + 2 * d->m);
  }
  if (p->kernel == MCPX_KERNEL_WAVE) wg_ok = false;
  if (p->kernel == MCPX_KERNEL_WORKGROUP) wave_ok = false;
  if (*mw || *band) wave_ok = true;
  if (!wave_ok && !wg_ok) {
    if (mod)
      return fail(MCPX_EUNSUPPORTED, "the generated module has no %s kernel for linear_solver=%d (n=%d m=%d)",
                  p->kernel == MCPX_KERNEL_WAVE ? "one-wave" : (p->kernel == MCPX_KERNEL_WORKGROUP ? "workgroup" : ""),
                  ls, d->n, d->m);
    return fail(MCPX_EUNSUPPORTED, "problem size n=%d m=%d, linear_solver=%d exceeds the kernels (one wave: "
                "reduced/schur n+m <= %d, dense n+2m <= %d; workgroup: reduced/dense n+2m <= %d, "
                "schur: QP family, n <= %d)",
                d->n, d->m, ls, MCPX_MAX_KKT_DIM, MCPX_MAX_KKT_DIM, MCPX_MAX_WG_KKT_DIM, mcpx::wg::kGjMax);
  }
  *wg = !wave_ok;
  if (!(p->tol > 0) || !(p->min_stepsize > 0) || !(p->decay > 0 && p->decay < 1) || std::isnan(p->tau) ||
      std::isnan(p->tightening_rate) || std::isnan(p->loosening_rate) || p->max_inner_iters < 1 ||
      p->max_outer_iters < 1)
    return fail(MCPX_EINVAL, "invalid solver parameters (tol>0, min_stepsize>0, 0<decay<1, iteration limits >= 1)");
  if (p->max_inner_iters > MCPX_MAX_INNER_ITERS)
    return fail(MCPX_EUNSUPPORTED, "max_inner_iters %d > %d", p->max_inner_iters, MCPX_MAX_INNER_ITERS);
  std::memset(a, 0, sizeof *a);
  a->n = d->n;
  a->m = d->m;
  a->solver = ls;
  a->family = d->family;
  a->theta_ld = d->theta_ld;
  a->max_inner = p->max_inner_iters;
  a->max_outer = p->max_outer_iters;
  a->tol = p->tol;
  a->decay = p->decay;
  a->c_tau = 1.0 - p->tau;  // src/solver.jl:129 (1 - τ)
  // src/solver.jl:128-135: trials α = 1, decay, decay², … until α < min_stepsize
  double al = 1.0;
  int e = 0;
  for (;;) {
    if (e >= MCPX_MAX_LS_TRIALS) return fail(MCPX_EUNSUPPORTED, "min_stepsize/decay need more than %d line-search trials", MCPX_MAX_LS_TRIALS);
    if (al < p->min_stepsize) break;
    al *= p->decay;
    ++e;
  }
  a->n_trials = e + 1;
  for (int k = 0; k <= p->max_inner_iters; ++k) {  // src/solver.jl:111-113
    a->tight[k] = 1.0 - std::exp(-p->tightening_rate * (double)k);
    a->loose[k] = 1.0 + std::exp(-p->loosening_rate * (double)k);
  }
  return MCPX_OK;
}

// ---- generated nonlinear modules ---------------------------------------------
constexpr int32_t kNLLayout = 4;  // mcpx_nl_meta[0] of csrc/ipm_nl_kernel.hpp
const char* const kNLKernel[3] = {"mcpx_nl_solve_reduced", "mcpx_nl_solve_dense", "mcpx_nl_solve_schur"};

// `mod` on device `dev` (the current device), loaded on first use.
int module_on(mcpx_module* mod, int dev, hipModule_t* hm) {
  std::lock_guard<std::mutex> lock(mod->mu);
  auto it = mod->loaded.find(dev);
  if (it != mod->loaded.end()) {
    *hm = it->second;
    return MCPX_OK;
  }
  HIP_TRY(hipModuleLoadData(hm, mod->image.data()));
  mod->loaded[dev] = *hm;
  return MCPX_OK;
}

// The module's kernel for linear solver `solver` (one-wave, or the workgroup
// kernel "<name>_wg") on the current device.
int nl_function(mcpx_module* mod, int solver, bool wg, hipFunction_t* f, bool mw = false) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  hipModule_t hm;
  const int rc = module_on(mod, dev, &hm);
  if (rc) return rc;
  const std::string name = std::string(kNLKernel[solver]) + (wg ? "_wg" : (mw ? "_mw" : ""));
  if (hipModuleGetFunction(f, hm, name.c_str()) != hipSuccess)
    return fail(MCPX_EUNSUPPORTED, "the generated module has no %s kernel", name.c_str());
  return MCPX_OK;
}

// Picks the kernel: a compile-time-(n, m) specialisation when one exists (and
// MCPX_GENERIC_KERNELS is not set), else the runtime-(n, m) kernel for nmax.
hipError_t launch(int nmax, const mcpx::KernelArgs& a, int64_t nb, hipStream_t st) {
  if (specialized_enabled()) {
    const hipError_t e = mcpx::launch_ipm_spec(a.family, a.solver, a.n, a.m, a, nb, st);
    if (e != hipErrorNotFound) return e;
  }
  const bool qp = a.family == MCPX_FAMILY_QP;
  switch (a.solver) {
    case MCPX_LINSOLVE_REDUCED:
      return qp ? mcpx::launch_ipm_red_qp(nmax, a, nb, st) : mcpx::launch_ipm_red_aff(nmax, a, nb, st);
    case MCPX_LINSOLVE_DENSE:
      return qp ? mcpx::launch_ipm_dense_qp(nmax, a, nb, st) : mcpx::launch_ipm_dense_aff(nmax, a, nb, st);
    default:
      return qp ? mcpx::launch_ipm_schur_qp(nmax, a, nb, st) : mcpx::launch_ipm_schur_aff(nmax, a, nb, st);
  }
}

// uint64 words of one instance's active-set mask: ⌈m/64⌉, at least 1 (include/mcpx.h)
inline int64_t mask_words(int m) { return m > 64 ? (m + 63) / 64 : 1; }

// Per-instance pointers of chunk [b0, b0 + nb) into the kernel args.
void set_chunk(mcpx::KernelArgs& a, const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
               const double* s0, const mcpx_out* o, int64_t b0) {
  const int n = d->n, m = d->m;
  a.theta = theta + b0 * d->theta_ld;
  a.x0 = x0 ? x0 + b0 * n : nullptr;
  a.y0 = y0 ? y0 + b0 * m : nullptr;
  a.s0 = s0 ? s0 + b0 * m : nullptr;
  a.x = o->x + b0 * n;
  a.y = o->y + b0 * m;
  a.s = o->s + b0 * m;
  a.kkt_error = o->kkt_error + b0;
  a.eps = o->eps + b0;
  a.outer_iters = o->outer_iters + b0;
  a.status = o->status + b0;
  a.newton_iters = o->newton_iters ? o->newton_iters + b0 : nullptr;
  a.active_mask = o->active_mask ? o->active_mask + b0 * mask_words(m) : nullptr;
  a.alpha_trace = (o->alpha_trace && o->trace_len > 0) ? o->alpha_trace + b0 * (int64_t)o->trace_len * 2 : nullptr;
  a.trace_len = o->alpha_trace ? o->trace_len : 0;
  a.fail_reason = o->fail_reason ? o->fail_reason + b0 : nullptr;
}

hipError_t dev_alloc(void** p, size_t bytes, hipStream_t st);  // the library's block cache (below)
void dev_release(void* p, hipStream_t st);

// Workgroup-per-instance launch (ipm_wg_impl.hpp): a persistent grid of the
// resident workgroups pulls instances from an atomic counter; each workgroup
// slot owns a workspace in HBM ([K | rhs] row-major, and for a generated module
// its Jacobian blocks), allocated stream-ordered for this call.
int launch_wg(const mcpx_desc* d, const double* theta, const double* x0, const double* y0, const double* s0,
              const mcpx_out* o, mcpx::KernelArgs a, int nv, hipStream_t st, mcpx_module* mod) {
  const int n = d->n, m = d->m, ls = a.solver;
  const int ns = ls == MCPX_LINSOLVE_SCHUR ? n : (ls == MCPX_LINSOLVE_REDUCED ? n + m : n + 2 * m);
  hipFunction_t f = nullptr;
  const void* kp = nullptr;
  int per_cu = 0;
  if (mod) {
    const int rc = nl_function(mod, ls, true, &f);
    if (rc) return rc;
    HIP_TRY(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, mcpx::wg::kThreads, 0));
  } else {
    kp = mcpx::ipm_wg_kernel(a.family, ls, nv, ns);
    if (!kp) return fail(MCPX_EUNSUPPORTED, "no workgroup kernel for family %d, linear_solver %d, dim %d", a.family, ls, nv);
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, mcpx::wg::kThreads, 0));
  }
  int dev = 0, cus = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t slots_max = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  auto align = [](int64_t v) { return (v + 31) / 32 * 32; };  // 256-B boundaries
  mcpx::wg::WgArgs w{};
  w.ld = ns + 1;
  w.off_blk = align((int64_t)ns * w.ld);
  w.off_aux = align(w.off_blk + (mod ? mod->meta[6] : 0));
  w.off_rd = w.off_aux;  // (R·D⁻¹ no longer kept: the SCHUR entries read R and D⁻¹ directly)
  w.slot_stride = align(w.off_aux + (ls == MCPX_LINSOLVE_SCHUR ? 4 * (int64_t)m : 0));
  const int64_t CH = (int64_t)1 << 30;
  const int64_t grid_max = std::min(slots_max, std::min(CH, d->batch));
  double* ws = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(grid_max * w.slot_stride) + 256;
  HIP_TRY(dev_alloc((void**)&ws, bytes, st));
  w.work = ws;
  w.counter = (int32_t*)(ws + grid_max * w.slot_stride);
  int rc = MCPX_OK;
  for (int64_t b0 = 0; b0 < d->batch && rc == MCPX_OK; b0 += CH) {
    const int64_t nb = std::min(CH, d->batch - b0);
    const int grid = (int)std::min(grid_max, nb);
    set_chunk(a, d, theta, x0, y0, s0, o, b0);
    w.k = a;
    w.batch = nb;
    hipError_t e = hipMemsetAsync(w.counter, 0, sizeof(int32_t), st);
    if (e == hipSuccess) {
      if (mod) {
        void* params[] = {&w};
        e = hipModuleLaunchKernel(f, (unsigned)grid, 1, 1, mcpx::wg::kThreads, 1, 1, 0, st, params, nullptr);
      } else {
        e = mcpx::launch_ipm_wg(a.family, ls, nv, ns, w, grid, st);
      }
    }
    if (e != hipSuccess) rc = fail(MCPX_EHIP, "workgroup solver launch failed: %s", hipGetErrorString(e));
  }
  dev_release(ws, st);
  return rc;
}

// The band SCHUR kernel of a generated module (ipm_nl_band.hpp): one wave per resident slot
// on the work queue of the workgroup kernels, no workspace (LDS and VGPRs only).
int launch_band(const mcpx_desc* d, const double* theta, const double* x0, const double* y0, const double* s0,
                const mcpx_out* o, mcpx::KernelArgs a, hipStream_t st, mcpx_module* mod) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  hipModule_t hm;
  int rc = module_on(mod, dev, &hm);
  if (rc) return rc;
  hipFunction_t f = nullptr;
  if (hipModuleGetFunction(&f, hm, "mcpx_nl_solve_band") != hipSuccess)
    return fail(MCPX_EUNSUPPORTED, "the generated module has no band kernel");
  int per_cu = 0, cus = 0;
  HIP_TRY(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 64, 0));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t slots_max = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  // the kernel's per-slot HBM workspace (its U rows when they exceed its VGPR budget, mcpx_nl_meta[9])
  const int64_t stride = ((int64_t)mod->meta[9] + 31) / 32 * 32;
  const int64_t grid_max = std::min(slots_max, std::min((int64_t)1 << 30, d->batch));
  double* ws = nullptr;
  HIP_TRY(dev_alloc((void**)&ws, sizeof(double) * (size_t)(grid_max * stride) + 256, st));
  int32_t* counter = (int32_t*)(ws + grid_max * stride);
  mcpx::wg::WgArgs w{};
  w.counter = counter;
  w.work = ws;
  w.slot_stride = stride;
  const int64_t CH = (int64_t)1 << 30;
  for (int64_t b0 = 0; b0 < d->batch && rc == MCPX_OK; b0 += CH) {
    const int64_t nb = std::min(CH, d->batch - b0);
    const int grid = (int)std::min(grid_max, nb);
    set_chunk(a, d, theta, x0, y0, s0, o, b0);
    w.k = a;
    w.batch = nb;
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(int32_t), st);
    if (e == hipSuccess) {
      void* params[] = {&w};
      e = hipModuleLaunchKernel(f, (unsigned)grid, 1, 1, 64, 1, 1, 0, st, params, nullptr);
    }
    if (e != hipSuccess) rc = fail(MCPX_EHIP, "band solver launch failed: %s", hipGetErrorString(e));
  }
  dev_release(ws, st);
  return rc;
}

int launch_chunks(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                  const double* s0, const mcpx_out* o, mcpx::KernelArgs a, int nmax, hipStream_t st,
                  mcpx_module* mod = nullptr, bool wg = false, bool mw = false, bool band = false) {
  if (band) return launch_band(d, theta, x0, y0, s0, o, a, st, mod);
  if (wg) return launch_wg(d, theta, x0, y0, s0, o, a, nmax, st, mod);
  hipFunction_t nlf = nullptr;  // generated module: its kernel, launched by hipModuleLaunchKernel
  if (mod) {
    const int rc = nl_function(mod, a.solver, false, &nlf, mw);
    if (rc) return rc;
  }
  const unsigned threads = mw ? 256 : 64;  // the multi-wave SCHUR kernel: 4 waves per instance
  const int64_t CH = (int64_t)1 << 30;
  for (int64_t b0 = 0; b0 < d->batch; b0 += CH) {
    const int64_t nb = std::min(CH, d->batch - b0);
    set_chunk(a, d, theta, x0, y0, s0, o, b0);
    if (mod) {
      void* params[] = {&a};
      HIP_TRY(hipModuleLaunchKernel(nlf, (unsigned)nb, 1, 1, threads, 1, 1, 0, st, params, nullptr));
    } else {
      HIP_TRY(launch(nmax, a, nb, st));
    }
  }
  return MCPX_OK;
}

bool outputs_ok(const mcpx_out* o) {
  return o && o->x && o->y && o->s && o->kkt_error && o->eps && o->outer_iters && o->status &&
         o->trace_len >= 0;
}

// Library-internal device buffers: a per-device cache of hipMalloc'd blocks, never unmapped.
// A block goes back to the cache with an event recorded on the stream of its last use; the
// next user (any stream of that device) takes it after a stream wait on that event, so reuse
// stays stream-ordered without host synchronisation.  (HIP 7.2's stream-ordered pools —
// hipMallocFromPoolAsync / hipFreeAsync, whose default VM heap remaps recycled memory — gave
// wrong answers here: from the fourth back-to-back host call on, ~15 of 1,024 T = 10 games
// every other call, with torch's bundled HIP 7.0 runtime or DEBUG_HIP_MEM_POOL_VMHEAP=0
// never; tools/band_stress.py)  Idle blocks beyond kCacheKeep bytes per
// device are freed once their last use has completed; the cache lives for the process (no
// HIP calls during teardown).
constexpr uint64_t kCacheKeep = 4ull << 30;

// MCPX_POISON=1 (debug): every block handed out is filled with 0xFF bytes (NaN doubles) up to
// the requested size, and the rest of the block (at least kCanary bytes) with the canary byte
// 0xA5.  At release the tail is read back and checked: a write past the requested size is
// reported on stderr ("MCPX_POISON canary") and counted (mcpx_debug_canary_violations), and a
// kernel result that depended on workspace read before it was written turns NaN or changes.
// Host synchronisation at every release: a diagnostic mode, not for timing.
constexpr size_t kCanary = 4096;
constexpr unsigned char kCanaryByte = 0xA5;
std::atomic<int64_t> g_canary_bad{0};

bool poison_on() {
  static const bool on = [] {
    const char* v = std::getenv("MCPX_POISON");
    return v && std::atoi(v) == 1;
  }();
  return on;
}

struct Block {
  void* p = nullptr;
  size_t bytes = 0;
  size_t req = 0;             // MCPX_POISON: the size requested by the current user
  hipEvent_t last = nullptr;  // recorded after the block's last use
  bool busy = false;
};

// MCPX_POISON: fill a block just handed out (stream-ordered)
hipError_t poison_block(Block& b, size_t bytes, hipStream_t st) {
  b.req = bytes;
  hipError_t e = hipMemsetAsync(b.p, 0xFF, bytes, st);
  if (e == hipSuccess) e = hipMemsetAsync((char*)b.p + bytes, kCanaryByte, b.bytes - bytes, st);
  return e;
}

// MCPX_POISON: check a block's tail after its last use on `st` (host-synchronising)
void check_canary(const Block& b, hipStream_t st) {
  const size_t tail = b.bytes - b.req;
  std::vector<unsigned char> h(tail);
  if (hipMemcpyAsync(h.data(), (const char*)b.p + b.req, tail, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    std::fprintf(stderr, "MCPX_POISON canary: could not read back block %p\n", b.p);
    g_canary_bad.fetch_add(1);
    return;
  }
  for (size_t i = 0; i < tail; ++i)
    if (h[i] != kCanaryByte) {
      std::fprintf(stderr, "MCPX_POISON canary: block %p (%zu bytes requested, %zu held) overwritten at +%zu\n",
                   b.p, b.req, b.bytes, b.req + i);
      g_canary_bad.fetch_add(1);
      return;
    }
}

struct BlockCache {
  std::mutex mu;
  std::map<int, std::vector<Block>> dev;  // device → blocks
};

BlockCache& block_cache() {
  static BlockCache* c = new BlockCache;  // never destroyed
  return *c;
}

hipError_t dev_alloc(void** p, size_t bytes, hipStream_t st) {
  *p = nullptr;
  int d = 0;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return e;
  const size_t need = std::max<size_t>(bytes, 1) + (poison_on() ? kCanary : 0);
  const size_t want = (need + (2u << 20) - 1) / (2u << 20) * (2u << 20);  // 2 MiB granules
  BlockCache& c = block_cache();
  std::lock_guard<std::mutex> lock(c.mu);
  auto& v = c.dev[d];
  Block* best = nullptr;  // the smallest idle block that fits without wasting more than half of it
  for (auto& b : v)
    if (!b.busy && b.bytes >= want && b.bytes <= 2 * want && (!best || b.bytes < best->bytes)) best = &b;
  if (best) {
    if (best->last && (e = hipStreamWaitEvent(st, best->last, 0)) != hipSuccess) return e;
    if (poison_on() && (e = poison_block(*best, bytes, st)) != hipSuccess) return e;
    best->busy = true;
    *p = best->p;
    return hipSuccess;
  }
  Block b;
  b.bytes = want;
  if ((e = hipMalloc(&b.p, want)) != hipSuccess) {
    // out of memory: free the idle blocks (after their last use) and try once more
    for (auto it = v.begin(); it != v.end();) {
      if (it->busy) { ++it; continue; }
      if (it->last) (void)hipEventSynchronize(it->last), (void)hipEventDestroy(it->last);
      (void)hipFree(it->p);
      it = v.erase(it);
    }
    (void)hipGetLastError();
    if ((e = hipMalloc(&b.p, want)) != hipSuccess) return e;
  }
  if (poison_on() && (e = poison_block(b, bytes, st)) != hipSuccess) return e;
  b.busy = true;
  v.push_back(b);
  *p = b.p;
  return hipSuccess;
}

void dev_release(void* p, hipStream_t st) {
  if (!p) return;
  BlockCache& c = block_cache();
  std::lock_guard<std::mutex> lock(c.mu);
  for (auto& [d, v] : c.dev) {
    for (auto& b : v) {
      if (b.p != p) continue;
      if (poison_on()) check_canary(b, st);
      if (!b.last) (void)hipEventCreateWithFlags(&b.last, hipEventDisableTiming);
      if (b.last) (void)hipEventRecord(b.last, st);
      b.busy = false;
      uint64_t idle = 0;  // trim: idle bytes beyond kCacheKeep, oldest first, once completed
      for (auto& q : v) idle += q.busy ? 0 : q.bytes;
      for (auto it = v.begin(); it != v.end() && idle > kCacheKeep;) {
        if (it->busy || it->p == p || (it->last && hipEventQuery(it->last) != hipSuccess)) { ++it; continue; }
        idle -= it->bytes;
        if (it->last) (void)hipEventDestroy(it->last);
        (void)hipFree(it->p);
        it = v.erase(it);
      }
      (void)d;
      return;
    }
  }
}

template <class T>
struct DevBuf {  // a cache block used on the null stream (synchronous callers)
  T* p = nullptr;
  ~DevBuf() { dev_release(p, nullptr); }
  hipError_t alloc(size_t count) { return count ? dev_alloc((void**)&p, count * sizeof(T), nullptr) : hipSuccess; }
};

template <class T>
struct AsyncBuf {  // a cache block, released on the stream it was allocated on
  T* p = nullptr;
  hipStream_t st = nullptr;
  hipError_t alloc(size_t count, hipStream_t s) {
    st = s;
    return count ? dev_alloc((void**)&p, count * sizeof(T), s) : hipSuccess;
  }
  ~AsyncBuf() { dev_release(p, st); }
};

// θ buffers the host-buffer pipeline rotates through: MCPX_HOST_BUFFERS (A/B knob, 2..8,
// default 3: chunk c+1 and c+2 upload while chunk c solves).
constexpr int kMaxHostBufs = 8;
int host_buffers() {
  const char* e = std::getenv("MCPX_HOST_BUFFERS");
  const int v = e ? std::atoi(e) : 3;
  return v < 2 ? 2 : (v > kMaxHostBufs ? kMaxHostBufs : v);
}

// Instances per pipelined chunk: MCPX_HOST_CHUNK (A/B knob, ≥ 1024, default 4096:
// profiles/r02/host_pipeline.jsonl).
int64_t host_chunk() {
  const char* e = std::getenv("MCPX_HOST_CHUNK");
  const long long v = e ? std::atoll(e) : 4096;
  return v < 1024 ? 1024 : v;
}

// The pipeline's two streams and per-buffer events.  Creating streams per call maps new
// hardware queues every time (≈10 ms per call: profiles/r02/host_pipeline_trace.txt), so
// they come from a process-wide free list per device: a call takes one Pipe and gives
// it back when it returns, concurrent calls get different ones (the ABI stays
// reentrant), and none is ever destroyed (no HIP calls during process teardown).
struct Pipe {
  hipStream_t up = nullptr, comp = nullptr;  // H→D uploads (serialised: full PCIe rate each), kernels
  hipEvent_t copied[kMaxHostBufs] = {}, consumed[kMaxHostBufs] = {};
  hipError_t init() {
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&up, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&comp, hipStreamNonBlocking)) != hipSuccess) return e;
    for (int k = 0; k < kMaxHostBufs; ++k) {
      if ((e = hipEventCreateWithFlags(&copied[k], hipEventDisableTiming)) != hipSuccess) return e;
      if ((e = hipEventCreateWithFlags(&consumed[k], hipEventDisableTiming)) != hipSuccess) return e;
    }
    return hipSuccess;
  }
  void destroy() {  // a Pipe whose init() failed part-way: release what it created
    for (int k = 0; k < kMaxHostBufs; ++k) {
      if (copied[k]) (void)hipEventDestroy(copied[k]);
      if (consumed[k]) (void)hipEventDestroy(consumed[k]);
    }
    if (up) (void)hipStreamDestroy(up);
    if (comp) (void)hipStreamDestroy(comp);
  }
};

std::mutex g_pipe_mu;
std::map<int, std::vector<Pipe*>> g_pipe_free;

struct PipeLease {  // a Pipe of device `dev` for the duration of one call (current device = dev)
  Pipe* p = nullptr;
  int dev = -1;
  int acquire(int d) {
    dev = d;
    {
      std::lock_guard<std::mutex> lock(g_pipe_mu);
      auto& v = g_pipe_free[d];
      if (!v.empty()) {
        p = v.back();
        v.pop_back();
        return MCPX_OK;
      }
    }
    Pipe* q = new Pipe;
    if (hipError_t e = q->init(); e != hipSuccess) {
      q->destroy();
      delete q;
      return fail(MCPX_EHIP, "stream setup: %s", hipGetErrorString(e));
    }
    p = q;
    return MCPX_OK;
  }
  ~PipeLease() {
    if (!p) return;
    std::lock_guard<std::mutex> lock(g_pipe_mu);
    g_pipe_free[dev].push_back(p);
  }
};

// One device's share of mcpx_solve_batch: instances [b0, b0+nb), pipelined in chunks
// of MCPX_HOST_CHUNK instances through NB rotating θ buffers.  θ (and warm starts) of
// every chunk go up on ONE upload stream, back to back at the full host-link rate; the
// compute stream runs chunk c once its upload is done (event), and the upload of chunk
// c + NB waits for chunk c's kernel to release its buffer (event).  Outputs land in
// whole-shard device buffers and come back once, after the last kernel.
int solve_shard(int dev, const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                const double* s0, const mcpx_params* prm, mcpx_out* o, int64_t b0, int64_t nb,
                mcpx_module* mod = nullptr) {
  HIP_TRY(hipSetDevice(dev));
  int rc = check_device(dev);
  if (rc) return rc;
  mcpx::KernelArgs a;
  int nmax;
  bool wg = false, mw = false, band = false;
  if ((rc = prepare(d, prm, &a, &nmax, mod, &wg, &mw, &band))) return rc;
  const int n = d->n, m = d->m;
  const int64_t W = mask_words(m);
  PipeLease lease;
  if ((rc = lease.acquire(dev))) return rc;
  Pipe* P = lease.p;
  const int NB = host_buffers();
  const int64_t ch = std::min(host_chunk(), nb);
  const int64_t ld = d->theta_ld;
  hipStream_t cs = P->comp, us = P->up;
  AsyncBuf<double> th[kMaxHostBufs], wx[kMaxHostBufs], wy[kMaxHostBufs], ws[kMaxHostBufs];
  AsyncBuf<double> x, y, s, kkt, eps;
  AsyncBuf<int32_t> outer, status, newton;
  AsyncBuf<uint64_t> am;
  AsyncBuf<uint8_t> tr, fr;
  // declared after the buffers, so it runs before their (stream-ordered) frees on every
  // exit: no upload or kernel may still target a buffer when it returns to the cache
  struct Drain {
    hipStream_t a, b;
    ~Drain() {
      (void)hipStreamSynchronize(a);
      (void)hipStreamSynchronize(b);
    }
  } drain{us, cs};
  const int nbuf = (int)std::min<int64_t>(NB, (nb + ch - 1) / std::max<int64_t>(ch, 1));
  for (int k = 0; k < nbuf; ++k) {  // every buffer lives on the compute stream (allocated, used, freed there)
    HIP_TRY(th[k].alloc((size_t)ch * ld, cs));
    if (x0) HIP_TRY(wx[k].alloc((size_t)ch * n, cs));
    if (y0) HIP_TRY(wy[k].alloc((size_t)ch * m, cs));
    if (s0) HIP_TRY(ws[k].alloc((size_t)ch * m, cs));
  }
  HIP_TRY(x.alloc((size_t)nb * n, cs)); HIP_TRY(y.alloc((size_t)nb * m, cs)); HIP_TRY(s.alloc((size_t)nb * m, cs));
  HIP_TRY(kkt.alloc(nb, cs)); HIP_TRY(eps.alloc(nb, cs)); HIP_TRY(outer.alloc(nb, cs));
  HIP_TRY(status.alloc(nb, cs));
  if (o->newton_iters) HIP_TRY(newton.alloc(nb, cs));
  if (o->active_mask) HIP_TRY(am.alloc((size_t)nb * W, cs));
  if (o->fail_reason) HIP_TRY(fr.alloc(nb, cs));
  const bool want_tr = o->alpha_trace && o->trace_len > 0;
  if (want_tr) {
    HIP_TRY(tr.alloc((size_t)nb * o->trace_len * 2, cs));
    HIP_TRY(hipMemsetAsync(tr.p, 254, (size_t)nb * o->trace_len * 2, cs));
  }
  // the allocations (compute stream) before the first upload into them
  HIP_TRY(hipEventRecord(P->consumed[0], cs));
  HIP_TRY(hipStreamWaitEvent(us, P->consumed[0], 0));
  for (int64_t c0 = 0, ci = 0; c0 < nb; c0 += ch, ++ci) {
    const int k = (int)(ci % nbuf);
    const int64_t cn = std::min(ch, nb - c0), g0 = b0 + c0;
    if (ci >= nbuf) HIP_TRY(hipStreamWaitEvent(us, P->consumed[k], 0));  // chunk ci - nbuf released buffer k
    HIP_TRY(hipMemcpyAsync(th[k].p, theta + g0 * ld, sizeof(double) * (size_t)cn * ld, hipMemcpyHostToDevice, us));
    if (x0) HIP_TRY(hipMemcpyAsync(wx[k].p, x0 + g0 * n, sizeof(double) * cn * n, hipMemcpyHostToDevice, us));
    if (y0) HIP_TRY(hipMemcpyAsync(wy[k].p, y0 + g0 * m, sizeof(double) * cn * m, hipMemcpyHostToDevice, us));
    if (s0) HIP_TRY(hipMemcpyAsync(ws[k].p, s0 + g0 * m, sizeof(double) * cn * m, hipMemcpyHostToDevice, us));
    HIP_TRY(hipEventRecord(P->copied[k], us));
    HIP_TRY(hipStreamWaitEvent(cs, P->copied[k], 0));
    mcpx_out od{};
    od.x = x.p + c0 * n; od.y = y.p + c0 * m; od.s = s.p + c0 * m; od.kkt_error = kkt.p + c0; od.eps = eps.p + c0;
    od.outer_iters = outer.p + c0; od.status = status.p + c0; od.newton_iters = newton.p ? newton.p + c0 : nullptr;
    od.active_mask = am.p ? am.p + c0 * W : nullptr;
    od.alpha_trace = want_tr ? tr.p + c0 * (int64_t)o->trace_len * 2 : nullptr;
    od.trace_len = want_tr ? o->trace_len : 0;
    od.fail_reason = fr.p ? fr.p + c0 : nullptr;
    mcpx_desc dd = *d;
    dd.batch = cn;
    if ((rc = launch_chunks(&dd, th[k].p, wx[k].p, wy[k].p, ws[k].p, &od, a, nmax, cs, mod, wg, mw, band))) return rc;
    HIP_TRY(hipEventRecord(P->consumed[k], cs));
  }
  HIP_TRY(hipStreamSynchronize(us));
  HIP_TRY(hipStreamSynchronize(cs));
  auto back = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
    return bytes ? hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) : hipSuccess;
  };
  HIP_TRY(back(o->x + b0 * n, x.p, sizeof(double) * nb * n));
  HIP_TRY(back(o->y + b0 * m, y.p, sizeof(double) * nb * m));
  HIP_TRY(back(o->s + b0 * m, s.p, sizeof(double) * nb * m));
  HIP_TRY(back(o->kkt_error + b0, kkt.p, sizeof(double) * nb));
  HIP_TRY(back(o->eps + b0, eps.p, sizeof(double) * nb));
  HIP_TRY(back(o->outer_iters + b0, outer.p, sizeof(int32_t) * nb));
  HIP_TRY(back(o->status + b0, status.p, sizeof(int32_t) * nb));
  if (o->newton_iters) HIP_TRY(back(o->newton_iters + b0, newton.p, sizeof(int32_t) * nb));
  if (o->active_mask) HIP_TRY(back(o->active_mask + b0 * W, am.p, sizeof(uint64_t) * nb * W));
  if (want_tr) HIP_TRY(back(o->alpha_trace + b0 * o->trace_len * 2, tr.p, (size_t)nb * o->trace_len * 2));
  if (o->fail_reason) HIP_TRY(back(o->fail_reason + b0, fr.p, (size_t)nb));
  return MCPX_OK;
}


// ---- sensitivities (src/AutoDiff.jl) ----------------------------------------

// How a sensitivity call runs: one wave per instance (QP / affine, n + 2m ≤ 64: the
// register kernels of sens_kernel_impl.hpp, `nmax` wide) or one workgroup per instance
// (larger QP / affine systems in the dimension bucket `nv`, and every generated module).
struct SensPlan {
  int nmax = 0;
  bool wg = false;
  int nv = 0;
  mcpx_module* mod = nullptr;
};

// Validates a sensitivity call; fills the scalar part of the args and the plan.
int prepare_sens(const mcpx_desc* d, mcpx::SensArgs* a, SensPlan* plan, bool jvp, mcpx_module* mod = nullptr) {
  if (!d) return fail(MCPX_EINVAL, "desc must be non-NULL");
  int64_t pd;
  if (mod) {
    if (d->family != MCPX_FAMILY_NONLINEAR)
      return fail(MCPX_EINVAL, "a generated module differentiates family MCPX_FAMILY_NONLINEAR (got %d)", d->family);
    if (d->n != mod->meta[1] || d->m != mod->meta[2])
      return fail(MCPX_EINVAL, "desc (n=%d, m=%d) does not match the module (n=%d, m=%d)", d->n, d->m,
                  mod->meta[1], mod->meta[2]);
    pd = mod->meta[3];
  } else {
    if (d->family == MCPX_FAMILY_NONLINEAR)
      return fail(MCPX_EINVAL, "family MCPX_FAMILY_NONLINEAR is differentiated through its generated module "
                  "(mcpx_vjp_batch_module / mcpx_jvp_batch_module)");
    pd = mcpx_theta_dim(d->family, d->n, d->m);
  }
  if (pd < 0) return fail(MCPX_EINVAL, "bad family %d or negative dimensions (n=%d, m=%d)", d->family, d->n, d->m);
  if (d->n + d->m < 1) return fail(MCPX_EINVAL, "empty problem (n = m = 0)");
  if (d->batch < 0) return fail(MCPX_EINVAL, "negative batch");
  if (d->theta_ld < pd) return fail(MCPX_EINVAL, "theta_ld %lld < parameter dimension %lld", (long long)d->theta_ld, (long long)pd);
  const int N = d->n + 2 * d->m;
  *plan = SensPlan{};
  plan->mod = mod;
  if (mod) {
    const int bit = jvp ? MCPX_MODULE_JVP : MCPX_MODULE_VJP;
    if (!((mod->meta[5] >> bit) & 1))
      return fail(MCPX_EUNSUPPORTED, "the generated module has no %s kernel (n=%d m=%d: its LDS footprint does not fit)",
                  jvp ? "JVP" : "VJP", d->n, d->m);
    plan->wg = true;
  } else if (N <= MCPX_MAX_KKT_DIM) {
    plan->nmax = pick_nmax(N);
  } else if (N <= MCPX_MAX_WG_KKT_DIM) {
    plan->wg = true;
    plan->nv = pick_wg_bucket(N);
  } else {
    return fail(MCPX_EUNSUPPORTED, "sensitivities need n + 2m <= %d (got n=%d m=%d)", MCPX_MAX_WG_KKT_DIM, d->n, d->m);
  }
  std::memset(a, 0, sizeof *a);
  a->theta_ld = d->theta_ld;
  a->p = pd;
  a->n = d->n;
  a->m = d->m;
  a->family = d->family;
  return MCPX_OK;
}

// Workgroup-per-instance sensitivity launch (sens_wg_impl.hpp): persistent grid of the
// resident workgroups on an atomic work queue, per-slot HBM workspace for [K | rhs]
// (and a module's Jacobian blocks and ∇F_θ), allocated stream-ordered for this call.
int launch_sens_wg_impl(bool jvp, const mcpx_desc* d, mcpx::SensArgs a, const SensPlan& plan, hipStream_t st) {
  const int n = d->n, m = d->m, N = n + 2 * m, nr = n + m;
  const int ns = jvp ? N : nr;
  const int K = a.n_partials;
  // (the condition estimate: two N-vectors of scratch in the right-hand-side area)
  const int nrhs = a.mode == 1 ? 2 : (jvp ? std::max(1, std::min(K, MCPX_JVP_RHS)) : 1);
  hipFunction_t f = nullptr;
  const void* kp = nullptr;
  int per_cu = 0;
  if (plan.mod) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipModule_t hm;
    const int rc = module_on(plan.mod, dev, &hm);
    if (rc) return rc;
    const char* name = jvp ? "mcpx_nl_jvp_wg" : "mcpx_nl_vjp_wg";
    if (hipModuleGetFunction(&f, hm, name) != hipSuccess)
      return fail(MCPX_EUNSUPPORTED, "the generated module has no %s kernel", name);
    HIP_TRY(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, mcpx::wg::kThreads, 0));
  } else {
    kp = mcpx::sens_wg_kernel(a.family, jvp, plan.nv);
    if (!kp) return fail(MCPX_EUNSUPPORTED, "no workgroup sensitivity kernel for family %d, dim %d", a.family, plan.nv);
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, mcpx::wg::kThreads, 0));
  }
  int dev = 0, cus = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t slots_max = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  auto align = [](int64_t v) { return (v + 31) / 32 * 32; };  // 256-B boundaries
  mcpx::wg::WgSensArgs w{};
  w.ld = ns + nrhs;
  w.nrhs = nrhs;
  w.off_blk = align((int64_t)ns * w.ld);
  w.off_dth = align(w.off_blk + (plan.mod ? plan.mod->meta[6] : 0));
  w.off_sol = align(w.off_dth + (plan.mod ? (int64_t)nr * a.p : 0));
  w.slot_stride = align(w.off_sol + (jvp ? (int64_t)nrhs * ns : 0));
  const int64_t CH = (int64_t)1 << 30;
  const int64_t grid_max = std::min(slots_max, std::min(CH, d->batch));
  double* ws = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(grid_max * w.slot_stride) + 256;
  HIP_TRY(dev_alloc((void**)&ws, bytes, st));
  w.work = ws;
  w.counter = (int32_t*)(ws + grid_max * w.slot_stride);
  int rc = MCPX_OK;
  for (int64_t b0 = 0; b0 < d->batch && rc == MCPX_OK; b0 += CH) {
    const int64_t nb = std::min(CH, d->batch - b0);
    const int grid = (int)std::min(grid_max, nb);
    w.s = a;
    w.s.theta = a.theta + b0 * d->theta_ld;
    w.s.x = a.x + b0 * n;
    w.s.y = a.y + b0 * m;
    w.s.s = a.s + b0 * m;
    w.s.gx = a.gx ? a.gx + b0 * n : nullptr;
    w.s.gy = a.gy ? a.gy + b0 * m : nullptr;
    w.s.gs = a.gs ? a.gs + b0 * m : nullptr;
    w.s.theta_dot = a.theta_dot ? a.theta_dot + b0 * K * a.p : nullptr;
    w.s.out = a.out + (a.mode == 1 ? b0 : (jvp ? b0 * K * N : b0 * a.p));
    w.s.status = a.status ? a.status + b0 : nullptr;
    w.batch = nb;
    hipError_t e = hipMemsetAsync(w.counter, 0, sizeof(int32_t), st);
    if (e == hipSuccess) {
      if (plan.mod) {
        void* params[] = {&w};
        e = hipModuleLaunchKernel(f, (unsigned)grid, 1, 1, mcpx::wg::kThreads, 1, 1, 0, st, params, nullptr);
      } else {
        e = mcpx::launch_sens_wg(a.family, jvp, plan.nv, w, grid, st);
      }
    }
    if (e != hipSuccess) rc = fail(MCPX_EHIP, "workgroup sensitivity launch failed: %s", hipGetErrorString(e));
  }
  dev_release(ws, st);
  return rc;
}

// Enqueue VJP (jvp = false) or JVP launches over the batch: the one-wave kernels in
// chunks of 2^30 instances, or the workgroup kernels.
int launch_sens(bool jvp, const mcpx_desc* d, mcpx::SensArgs a, const SensPlan& plan, const double* theta,
                const double* x, const double* y, const double* s, const double* gx, const double* gy,
                const double* gs, const double* tdot, double* out, int32_t* status, hipStream_t st) {
  if (plan.wg) {
    a.theta = theta;
    a.x = x;
    a.y = y;
    a.s = s;
    a.gx = gx;
    a.gy = gy;
    a.gs = gs;
    a.theta_dot = tdot;
    a.out = out;
    a.status = status;
    return launch_sens_wg_impl(jvp, d, a, plan, st);
  }
  const int64_t CH = (int64_t)1 << 30;
  const int n = d->n, m = d->m, N = n + 2 * m, K = a.n_partials;
  for (int64_t b0 = 0; b0 < d->batch; b0 += CH) {
    const int64_t nb = std::min(CH, d->batch - b0);
    a.theta = theta + b0 * d->theta_ld;
    a.x = x + b0 * n;
    a.y = y + b0 * m;
    a.s = s + b0 * m;
    a.gx = gx ? gx + b0 * n : nullptr;
    a.gy = gy ? gy + b0 * m : nullptr;
    a.gs = gs ? gs + b0 * m : nullptr;
    a.theta_dot = tdot ? tdot + b0 * K * a.p : nullptr;
    a.out = out + (jvp ? b0 * K * N : b0 * a.p);
    a.status = status ? status + b0 : nullptr;
    // the VJP factors the slack-eliminated (n+m)-dim system, the JVP the full n+2m
    HIP_TRY(jvp ? mcpx::launch_jvp(plan.nmax, a, nb, st) : mcpx::launch_vjp(pick_nmax(n + m), a, nb, st));
  }
  return MCPX_OK;
}

// One device's share [b0, b0+nb) of a host-buffer sensitivity call.
int sens_shard(bool jvp, int dev, const mcpx_desc* d, const mcpx::SensArgs& a0, const SensPlan& plan,
               const double* theta, const double* x, const double* y, const double* s, const double* gx,
               const double* gy, const double* gs, const double* tdot, double* out, int32_t* status, int64_t b0,
               int64_t nb) {
  HIP_TRY(hipSetDevice(dev));
  int rc = check_device(dev);
  if (rc) return rc;
  const int n = d->n, m = d->m, N = n + 2 * m, K = a0.n_partials;
  const int64_t p = a0.p;
  DevBuf<double> th, dx, dy, ds, dgx, dgy, dgs, dtd, dout;
  DevBuf<int32_t> dst;
  auto up = [&](DevBuf<double>& b, const double* h, size_t per) -> hipError_t {
    if (!h || !per || !nb) return hipSuccess;
    hipError_t e = b.alloc((size_t)nb * per);
    return e != hipSuccess ? e : hipMemcpy(b.p, h + b0 * per, sizeof(double) * nb * per, hipMemcpyHostToDevice);
  };
  HIP_TRY(up(th, theta, (size_t)d->theta_ld));
  HIP_TRY(up(dx, x, n)); HIP_TRY(up(dy, y, m)); HIP_TRY(up(ds, s, m));
  HIP_TRY(up(dgx, gx, n)); HIP_TRY(up(dgy, gy, m)); HIP_TRY(up(dgs, gs, m));
  HIP_TRY(up(dtd, tdot, (size_t)K * p));
  const size_t per_out = a0.mode == 1 ? 1 : (jvp ? (size_t)K * N : (size_t)p);
  HIP_TRY(dout.alloc((size_t)nb * per_out));
  if (status) HIP_TRY(dst.alloc(nb));
  mcpx_desc dd = *d;
  dd.batch = nb;
  // empty x/y blocks (n = 0 or m = 0) still need a valid base pointer
  const double* bx = dx.p ? dx.p : th.p;
  const double* by = dy.p ? dy.p : th.p;
  const double* bs = ds.p ? ds.p : th.p;
  // an empty output (p = 0, or K = 0) still needs a valid base pointer
  double* bo = dout.p ? dout.p : (double*)th.p;
  if ((rc = launch_sens(jvp, &dd, a0, plan, th.p, bx, by, bs, gx ? dgx.p : nullptr, gy ? dgy.p : nullptr,
                        gs ? dgs.p : nullptr, dtd.p, bo, status ? dst.p : nullptr, nullptr))) {
    (void)hipDeviceSynchronize();  // nothing may still run on the buffers freed on return
    return rc;
  }
  HIP_TRY(hipDeviceSynchronize());
  if (per_out) HIP_TRY(hipMemcpy(out + b0 * per_out, dout.p, sizeof(double) * nb * per_out, hipMemcpyDeviceToHost));
  if (status) HIP_TRY(hipMemcpy(status + b0, dst.p, sizeof(int32_t) * nb, hipMemcpyDeviceToHost));
  return MCPX_OK;
}

// Shards of a host-buffer call: one per device, or MCPX_HOST_SHARDS = k contiguous shards
// over the caller's (clamped) devices round-robin — shard g runs on device g mod
// num_devices, never on a device the caller did not ask for (one host thread each; a test
// knob that runs the multi-device path on a box with fewer devices).
int host_shards(int num_devices, int64_t batch) {
  const char* e = std::getenv("MCPX_HOST_SHARDS");
  const int k = e ? std::atoi(e) : 0;
  if (k <= 0) return num_devices;
  return (int)std::max<int64_t>(1, std::min<int64_t>(k, batch));
}

// Host-buffer entry shared by mcpx_vjp_batch / mcpx_jvp_batch (and the module variants):
// contiguous shards, one thread per device.
int sens_host(bool jvp, const mcpx_desc* d, const mcpx::SensArgs& a, const SensPlan& plan, const double* theta,
              const double* x, const double* y, const double* s, const double* gx, const double* gy,
              const double* gs, const double* tdot, int num_devices, double* out, int32_t* status) {
  const int avail = mcpx_device_count();
  if (avail < 1) return fail(MCPX_ENODEV, "no HIP device visible");
  if (num_devices <= 0 || num_devices > avail) num_devices = avail;
  if ((int64_t)num_devices > d->batch) num_devices = (int)d->batch;
  const int devs = num_devices;
  num_devices = host_shards(devs, d->batch);
  std::vector<int64_t> start(num_devices + 1, 0);
  for (int g = 0; g < num_devices; ++g)
    start[g + 1] = start[g] + d->batch / num_devices + (g < d->batch % num_devices ? 1 : 0);
  std::vector<int> rcs(num_devices, 0);
  std::vector<std::string> errs(num_devices);
  std::vector<std::thread> th;
  for (int g = 0; g < num_devices; ++g)
    th.emplace_back([&, g] {
      rcs[g] = sens_shard(jvp, g % devs, d, a, plan, theta, x, y, s, gx, gy, gs, tdot, out, status, start[g],
                          start[g + 1] - start[g]);
      if (rcs[g]) errs[g] = g_err;
    });
  for (auto& t : th) t.join();
  for (int g = 0; g < num_devices; ++g)
    if (rcs[g]) return fail(rcs[g], "device %d: %s", g, errs[g].c_str());
  return MCPX_OK;
}

int sens_inputs_ok(const mcpx_desc* d, const double* theta, const double* x, const double* y, const double* s,
                   const double* out) {
  if (!theta || !out) return fail(MCPX_EINVAL, "theta and the output array must be non-NULL");
  if ((d->n > 0 && !x) || (d->m > 0 && (!y || !s))) return fail(MCPX_EINVAL, "solution arrays x/y/s must be non-NULL");
  return MCPX_OK;
}

int vjp_device_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                    const double* s, const double* gx, const double* gy, const double* gs, double* dtheta,
                    int32_t* status, void* stream) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_sens(d, &a, &plan, false, mod))) return rc;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, dtheta))) return rc;
  int dev = 0;
  if ((rc = current_device(&dev))) return rc;
  return launch_sens(false, d, a, plan, theta, x ? x : theta, y ? y : theta, s ? s : theta, gx, gy, gs, nullptr,
                     dtheta, status, (hipStream_t)stream);
}

int vjp_host_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                  const double* s, const double* gx, const double* gy, const double* gs, int num_devices,
                  double* dtheta, int32_t* status) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_sens(d, &a, &plan, false, mod))) return rc;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, dtheta))) return rc;
  return sens_host(false, d, a, plan, theta, x, y, s, gx, gy, gs, nullptr, num_devices, dtheta, status);
}

int jvp_device_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                    const double* s, int32_t n_partials, const double* theta_dot, double* zdot, int32_t* status,
                    void* stream) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_sens(d, &a, &plan, true, mod))) return rc;
  if (n_partials < 0) return fail(MCPX_EINVAL, "negative n_partials");
  a.n_partials = n_partials;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, zdot))) return rc;
  if (n_partials > 0 && !theta_dot) return fail(MCPX_EINVAL, "theta_dot is NULL");
  int dev = 0;
  if ((rc = current_device(&dev))) return rc;
  return launch_sens(true, d, a, plan, theta, x ? x : theta, y ? y : theta, s ? s : theta, nullptr, nullptr,
                     nullptr, theta_dot, zdot, status, (hipStream_t)stream);
}

int jvp_host_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                  const double* s, int32_t n_partials, const double* theta_dot, int num_devices, double* zdot,
                  int32_t* status) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_sens(d, &a, &plan, true, mod))) return rc;
  if (n_partials < 0) return fail(MCPX_EINVAL, "negative n_partials");
  a.n_partials = n_partials;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, zdot))) return rc;
  if (n_partials > 0 && !theta_dot) return fail(MCPX_EINVAL, "theta_dot is NULL");
  return sens_host(true, d, a, plan, theta, x, y, s, nullptr, nullptr, nullptr, theta_dot, num_devices, zdot,
                   status);
}

// mcpx_cond_batch*: the JVP workgroup kernels in their condition-estimate mode (every size and
// family runs the workgroup layout: the estimate's solves reuse the factors in the slot).
int prepare_cond(const mcpx_desc* d, mcpx::SensArgs* a, SensPlan* plan, mcpx_module* mod) {
  int rc = prepare_sens(d, a, plan, true, mod);
  if (rc) return rc;
  if (!plan->wg) {
    plan->wg = true;
    plan->nv = pick_wg_bucket(d->n + 2 * d->m);
  }
  a->mode = 1;
  return MCPX_OK;
}

int cond_device_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                     const double* s, double* rcond, int32_t* status, void* stream) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_cond(d, &a, &plan, mod))) return rc;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, rcond))) return rc;
  int dev = 0;
  if ((rc = current_device(&dev))) return rc;
  return launch_sens(true, d, a, plan, theta, x ? x : theta, y ? y : theta, s ? s : theta, nullptr, nullptr,
                     nullptr, nullptr, rcond, status, (hipStream_t)stream);
}

int cond_host_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x, const double* y,
                   const double* s, int num_devices, double* rcond, int32_t* status) {
  mcpx::SensArgs a;
  SensPlan plan;
  int rc;
  if ((rc = prepare_cond(d, &a, &plan, mod))) return rc;
  if (d->batch == 0) return MCPX_OK;
  if ((rc = sens_inputs_ok(d, theta, x, y, s, rcond))) return rc;
  return sens_host(true, d, a, plan, theta, x, y, s, nullptr, nullptr, nullptr, nullptr, num_devices, rcond, status);
}

// mcpx_solve_batch_device / mcpx_solve_batch_module_device (mod = nullptr: QP / affine kernels).
int solve_device_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x0,
                      const double* y0, const double* s0, const mcpx_params* prm, const mcpx_out* o,
                      void* stream) {
  mcpx::KernelArgs a;
  int nmax;
  bool wg = false, mw = false, band = false;
  int rc = prepare(d, prm, &a, &nmax, mod, &wg, &mw, &band);
  if (rc) return rc;
  if (!outputs_ok(o)) return fail(MCPX_EINVAL, "required output arrays missing");
  if (d->batch == 0) return MCPX_OK;
  if (!theta) return fail(MCPX_EINVAL, "theta is NULL");
  int dev = 0;
  if ((rc = current_device(&dev))) return rc;
  return launch_chunks(d, theta, x0, y0, s0, o, a, nmax, (hipStream_t)stream, mod, wg, mw, band);
}

// mcpx_solve_vjp_batch_device: the solve kernels with the pullback in their epilogue
// (ipm_inst_fused.hip) where they exist, else the solve then the VJP launches.
int solve_vjp_device_impl(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                          const double* s0, const mcpx_params* prm, const mcpx_out* o, const mcpx_cotangent* ct,
                          double* dtheta, int32_t* vstat, void* stream) {
  mcpx::KernelArgs a;
  int nmax;
  bool wg = false;
  int rc = prepare(d, prm, &a, &nmax, nullptr, &wg);
  if (rc) return rc;
  mcpx::SensArgs sa;
  SensPlan plan;
  if ((rc = prepare_sens(d, &sa, &plan, false))) return rc;
  if (!outputs_ok(o)) return fail(MCPX_EINVAL, "required output arrays missing");
  if (!ct) return fail(MCPX_EINVAL, "the cotangent must be non-NULL");
  if (d->batch == 0) return MCPX_OK;
  if (!theta || !dtheta) return fail(MCPX_EINVAL, "theta and dtheta must be non-NULL");
  int dev = 0;
  if ((rc = current_device(&dev))) return rc;
  const hipStream_t st = (hipStream_t)stream;
  const int n = d->n, m = d->m;
  if (!wg && specialized_enabled() && mcpx::has_fused_vjp(a.family, a.solver, n, m)) {
    const int64_t CH = (int64_t)1 << 30;
    a.ct_ax = ct->ax;
    a.ct_ay = ct->ay;
    a.ct_as = ct->as;
    for (int64_t b0 = 0; b0 < d->batch; b0 += CH) {
      const int64_t nb = std::min(CH, d->batch - b0);
      set_chunk(a, d, theta, x0, y0, s0, o, b0);
      a.vjp_dtheta = dtheta + b0 * sa.p;
      a.vjp_status = vstat ? vstat + b0 : nullptr;
      a.ct_bx = ct->bx ? ct->bx + b0 * n : nullptr;
      a.ct_by = ct->by ? ct->by + b0 * m : nullptr;
      a.ct_bs = ct->bs ? ct->bs + b0 * m : nullptr;
      HIP_TRY(mcpx::launch_ipm_fused_vjp(a.family, a.solver, n, m, a, nb, st));
    }
    return MCPX_OK;
  }
  if ((rc = launch_chunks(d, theta, x0, y0, s0, o, a, nmax, st, nullptr, wg))) return rc;
  sa.ga_x = ct->ax;
  sa.ga_y = ct->ay;
  sa.ga_s = ct->as;
  return launch_sens(false, d, sa, plan, theta, o->x, o->y, o->s, ct->bx, ct->by, ct->bs, nullptr, dtheta, vstat, st);
}

// mcpx_solve_batch / mcpx_solve_batch_module: contiguous shards, one host thread per device.
int solve_host_impl(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x0,
                    const double* y0, const double* s0, const mcpx_params* prm, int num_devices,
                    mcpx_out* o) {
  mcpx::KernelArgs a;
  int nmax;
  int rc = prepare(d, prm, &a, &nmax, mod);
  if (rc) return rc;
  if (!outputs_ok(o)) return fail(MCPX_EINVAL, "required output arrays missing");
  if (d->batch == 0) return MCPX_OK;
  if (!theta) return fail(MCPX_EINVAL, "theta is NULL");
  const int avail = mcpx_device_count();
  if (avail < 1) return fail(MCPX_ENODEV, "no HIP device visible");
  if (num_devices <= 0 || num_devices > avail) num_devices = avail;
  if ((int64_t)num_devices > d->batch) num_devices = (int)d->batch;
  const int devs = num_devices;
  num_devices = host_shards(devs, d->batch);
  // contiguous shards: shard g (device g mod devs) gets ⌊B/G⌋ (+1 for g < B mod G)
  std::vector<int64_t> start(num_devices + 1, 0);
  for (int g = 0; g < num_devices; ++g)
    start[g + 1] = start[g] + d->batch / num_devices + (g < d->batch % num_devices ? 1 : 0);
  if (num_devices == 1) return solve_shard(0, d, theta, x0, y0, s0, prm, o, 0, d->batch, mod);
  std::vector<int> rcs(num_devices, 0);
  std::vector<std::string> errs(num_devices);
  std::vector<std::thread> th;
  for (int g = 0; g < num_devices; ++g)
    th.emplace_back([&, g] {
      rcs[g] = solve_shard(g % devs, d, theta, x0, y0, s0, prm, o, start[g], start[g + 1] - start[g], mod);
      if (rcs[g]) errs[g] = g_err;
    });
  for (auto& t : th) t.join();
  for (int g = 0; g < num_devices; ++g)
    if (rcs[g]) return fail(rcs[g], "device %d: %s", g, errs[g].c_str());
  return MCPX_OK;
}

}  // namespace

extern "C" {

int mcpx_version(void) { return MCPX_VERSION; }

const char* mcpx_last_error(void) { return g_err.c_str(); }

void mcpx_default_params(mcpx_params* p) {
  if (!p) return;
  p->tol = 1e-4;              // src/solver.jl:42
  p->max_inner_iters = 20;    // :43
  p->max_outer_iters = 50;    // :44
  p->tightening_rate = 0.1;   // :45
  p->loosening_rate = 0.5;    // :46
  p->min_stepsize = 1e-4;     // :48
  p->tau = 0.995;             // :127
  p->decay = 0.5;             // :127
  p->linear_solver = MCPX_LINSOLVE_REDUCED;
  p->kernel = MCPX_KERNEL_AUTO;
}

int64_t mcpx_theta_dim(int32_t family, int32_t n, int32_t m) {
  if (n < 0 || m < 0) return -1;
  if (family == MCPX_FAMILY_QP) return (int64_t)n * n + (int64_t)m * n + m + n;
  if (family == MCPX_FAMILY_AFFINE) return (int64_t)n * n + 2 * (int64_t)n * m + (int64_t)m * m + n + m;
  return -1;
}

int mcpx_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int64_t mcpx_debug_canary_violations(void) { return g_canary_bad.load(); }

int mcpx_solve_batch_device(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                            const double* s0, const mcpx_params* prm, const mcpx_out* o, void* stream) {
  return solve_device_impl(nullptr, d, theta, x0, y0, s0, prm, o, stream);
}

int mcpx_solve_vjp_batch_device(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                                const double* s0, const mcpx_params* prm, const mcpx_out* out,
                                const mcpx_cotangent* ct, double* dtheta, int32_t* vjp_status, void* stream) {
  return solve_vjp_device_impl(d, theta, x0, y0, s0, prm, out, ct, dtheta, vjp_status, stream);
}

int mcpx_solve_batch(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                     const double* s0, const mcpx_params* prm, int num_devices, mcpx_out* o) {
  return solve_host_impl(nullptr, d, theta, x0, y0, s0, prm, num_devices, o);
}

int mcpx_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return fail(MCPX_EINVAL, "mcpx_host_register: NULL pointer or empty range");
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterPortable));
  return MCPX_OK;
}

int mcpx_host_unregister(void* ptr) {
  if (!ptr) return fail(MCPX_EINVAL, "mcpx_host_unregister: NULL pointer");
  HIP_TRY(hipHostUnregister(ptr));
  return MCPX_OK;
}

int mcpx_vjp_batch_device(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                          const double* s, const double* gx, const double* gy, const double* gs, double* dtheta,
                          int32_t* status, void* stream) {
  return vjp_device_impl(nullptr, d, theta, x, y, s, gx, gy, gs, dtheta, status, stream);
}

int mcpx_vjp_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y, const double* s,
                   const double* gx, const double* gy, const double* gs, int num_devices, double* dtheta,
                   int32_t* status) {
  return vjp_host_impl(nullptr, d, theta, x, y, s, gx, gy, gs, num_devices, dtheta, status);
}

int mcpx_jvp_batch_device(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                          const double* s, int32_t n_partials, const double* theta_dot, double* zdot,
                          int32_t* status, void* stream) {
  return jvp_device_impl(nullptr, d, theta, x, y, s, n_partials, theta_dot, zdot, status, stream);
}

int mcpx_jvp_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y, const double* s,
                   int32_t n_partials, const double* theta_dot, int num_devices, double* zdot, int32_t* status) {
  return jvp_host_impl(nullptr, d, theta, x, y, s, n_partials, theta_dot, num_devices, zdot, status);
}

int mcpx_cond_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y, const double* s,
                    int num_devices, double* rcond, int32_t* status) {
  return cond_host_impl(nullptr, d, theta, x, y, s, num_devices, rcond, status);
}

int mcpx_cond_batch_device(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                           const double* s, double* rcond, int32_t* status, void* stream) {
  return cond_device_impl(nullptr, d, theta, x, y, s, rcond, status, stream);
}

int mcpx_cond_batch_module(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                           const double* y, const double* s, int num_devices, double* rcond, int32_t* status) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return cond_host_impl(mod, d, theta, x, y, s, num_devices, rcond, status);
}

int mcpx_cond_batch_module_device(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                                  const double* y, const double* s, double* rcond, int32_t* status, void* stream) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return cond_device_impl(mod, d, theta, x, y, s, rcond, status, stream);
}

int mcpx_vjp_batch_module(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                          const double* y, const double* s, const double* gx, const double* gy, const double* gs,
                          int num_devices, double* dtheta, int32_t* status) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return vjp_host_impl(mod, d, theta, x, y, s, gx, gy, gs, num_devices, dtheta, status);
}

int mcpx_vjp_batch_module_device(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                                 const double* y, const double* s, const double* gx, const double* gy,
                                 const double* gs, double* dtheta, int32_t* status, void* stream) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return vjp_device_impl(mod, d, theta, x, y, s, gx, gy, gs, dtheta, status, stream);
}

int mcpx_jvp_batch_module(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                          const double* y, const double* s, int32_t n_partials, const double* theta_dot,
                          int num_devices, double* zdot, int32_t* status) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return jvp_host_impl(mod, d, theta, x, y, s, n_partials, theta_dot, num_devices, zdot, status);
}

int mcpx_jvp_batch_module_device(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x,
                                 const double* y, const double* s, int32_t n_partials, const double* theta_dot,
                                 double* zdot, int32_t* status, void* stream) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return jvp_device_impl(mod, d, theta, x, y, s, n_partials, theta_dot, zdot, status, stream);
}

// ---- generated nonlinear modules (MCPX_FAMILY_NONLINEAR) ----------------------

int mcpx_solve_batch_module(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x0,
                            const double* y0, const double* s0, const mcpx_params* prm, int num_devices,
                            mcpx_out* o) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return solve_host_impl(mod, d, theta, x0, y0, s0, prm, num_devices, o);
}

int mcpx_solve_batch_module_device(mcpx_module* mod, const mcpx_desc* d, const double* theta, const double* x0,
                                   const double* y0, const double* s0, const mcpx_params* prm,
                                   const mcpx_out* o, void* stream) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  return solve_device_impl(mod, d, theta, x0, y0, s0, prm, o, stream);
}

int mcpx_module_load(const char* path, mcpx_module** out) {
  if (!path || !out) return fail(MCPX_EINVAL, "path and out must be non-NULL");
  *out = nullptr;
  std::vector<char> img;
  {
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(MCPX_EINVAL, "cannot open code object '%s'", path);
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) img.insert(img.end(), buf, buf + k);
    std::fclose(f);
  }
  if (img.empty()) return fail(MCPX_EINVAL, "code object '%s' is empty", path);
  if (mcpx_device_count() < 1) return fail(MCPX_ENODEV, "no HIP device visible");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int rc = check_device(dev);
  if (rc) return rc;
  std::unique_ptr<mcpx_module> mod(new mcpx_module);
  mod->image = std::move(img);
  hipModule_t hm;
  if ((rc = module_on(mod.get(), dev, &hm))) return rc;
  hipDeviceptr_t dp = nullptr;
  size_t bytes = 0;
  if (hipModuleGetGlobal(&dp, &bytes, hm, "mcpx_nl_meta") != hipSuccess || bytes != sizeof mod->meta) {
    (void)hipModuleUnload(hm);
    return fail(MCPX_EINVAL, "'%s' is not an mcpx nonlinear module (no mcpx_nl_meta)", path);
  }
  HIP_TRY(hipMemcpyDtoH(mod->meta, dp, bytes));
  if (mod->meta[0] != kNLLayout) {
    (void)hipModuleUnload(hm);
    return fail(MCPX_EINVAL, "module layout version %d, this library expects %d", mod->meta[0], kNLLayout);
  }
  *out = mod.release();
  return MCPX_OK;
}

int mcpx_module_dims(const mcpx_module* mod, int32_t* n, int32_t* m, int32_t* p, int32_t* solvers) {
  if (!mod) return fail(MCPX_EINVAL, "module is NULL");
  if (n) *n = mod->meta[1];
  if (m) *m = mod->meta[2];
  if (p) *p = mod->meta[3];
  if (solvers) *solvers = mod->meta[5];
  return MCPX_OK;
}

void mcpx_module_unload(mcpx_module* mod) {
  if (!mod) return;
  int prev = 0;
  const bool have = hipGetDevice(&prev) == hipSuccess;
  for (auto& kv : mod->loaded)
    if (hipSetDevice(kv.first) == hipSuccess) (void)hipModuleUnload(kv.second);
  if (have) (void)hipSetDevice(prev);
  delete mod;
}

}  // extern "C"
