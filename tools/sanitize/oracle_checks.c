/* Sanitizer driver of the C oracle (oracle/ipm_oracle.c, built here with
 * -fsanitize=address,undefined): the README QP of the reference
 * (README.md:51-66, θ = [−0.5, 0.5]: x* = [1, 1], y* = [3.5, 2.5]) under every
 * linear solver, a batch of random QPs on several threads, degenerate inputs
 * (NaN θ, m = 0) and the sensitivity entry points.  Built by tools/sanitize/run.sh. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mcpx.h"

int oracle_solve_batch(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                       const double* s0, const mcpx_params* p, mcpx_out* o, int nthreads);
int oracle_vjp_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y, const double* s,
                     const double* gx, const double* gy, const double* gs, double* dtheta, int32_t* status,
                     int nthreads);

static int failures = 0;
#define EXPECT(c) do { if (!(c)) { fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); ++failures; } } while (0)

static void params(mcpx_params* p, int ls) {
  memset(p, 0, sizeof *p);
  p->tol = 1e-6; p->tightening_rate = 0.1; p->loosening_rate = 0.5; p->min_stepsize = 1e-4;
  p->tau = 0.995; p->decay = 0.5; p->max_inner_iters = 20; p->max_outer_iters = 50; p->linear_solver = ls;
}

typedef struct { double *x, *y, *s, *kkt, *eps; int32_t *outer, *status, *newton; uint64_t* am; uint8_t* tr; } bufs;

static mcpx_out alloc_out(int B, int n, int m, bufs* b) {
  b->x = calloc((size_t)B * (n ? n : 1), 8); b->y = calloc((size_t)B * (m ? m : 1), 8); b->s = calloc((size_t)B * (m ? m : 1), 8);
  b->kkt = calloc(B, 8); b->eps = calloc(B, 8); b->outer = calloc(B, 4); b->status = calloc(B, 4);
  b->newton = calloc(B, 4); b->am = calloc(B, 8); b->tr = calloc((size_t)B * 64 * 2, 1);
  mcpx_out o = {b->x, b->y, b->s, b->kkt, b->eps, b->outer, b->status, b->newton, b->am, b->tr, 64, 0};
  return o;
}
static void free_out(bufs* b) {
  free(b->x); free(b->y); free(b->s); free(b->kkt); free(b->eps); free(b->outer); free(b->status); free(b->newton);
  free(b->am); free(b->tr);
}

int main(void) {
  /* README QP: M = [2 1; 1 2], A = I, b = 1, θ = ϕ = [−0.5, 0.5] */
  const double thr[12] = {2, 1, 1, 2, 1, 0, 0, 1, 1, 1, -0.5, 0.5}; /* vec(M); vec(A); b; ϕ */
  for (int ls = 0; ls < 3; ++ls) {
    mcpx_params p; params(&p, ls);
    bufs b; mcpx_out o = alloc_out(1, 2, 2, &b);
    mcpx_desc d = {MCPX_FAMILY_QP, 2, 2, 0, 1, 12};
    EXPECT(oracle_solve_batch(&d, thr, NULL, NULL, NULL, &p, &o, 1) == 0);
    EXPECT(b.status[0] == 0 && fabs(b.x[0] - 1) < 1e-3 && fabs(b.y[0] - 3.5) < 1e-3 && b.am[0] == 3u);
    free_out(&b);
  }
  /* random QPs (n = 12, m = 7), 4 threads, every solver, plus the VJP */
  const int n = 12, m = 7, B = 64, P = n * n + m * n + m + n;
  double* theta = malloc(sizeof(double) * B * P);
  srand(7);
  for (int bi = 0; bi < B; ++bi) {
    double* t = theta + (size_t)bi * P;
    double Pm[12 * 12];
    for (int i = 0; i < n * n; ++i) Pm[i] = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double acc = i == j ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) acc += Pm[k * n + i] * Pm[k * n + j];
        t[j * n + i] = acc;
      }
    for (int i = n * n; i < P; ++i) t[i] = (double)rand() / RAND_MAX - 0.5;
  }
  theta[3] = NAN; /* instance 0: NaN θ → NaN kkt, never a crash */
  for (int ls = 0; ls < 3; ++ls) {
    mcpx_params p; params(&p, ls);
    bufs b; mcpx_out o = alloc_out(B, n, m, &b);
    mcpx_desc d = {MCPX_FAMILY_QP, n, m, 0, B, P};
    EXPECT(oracle_solve_batch(&d, theta, NULL, NULL, NULL, &p, &o, 4) == 0);
    int solved = 0;
    for (int i = 1; i < B; ++i) solved += b.status[i] == 0;
    EXPECT(solved == B - 1);
    EXPECT(isnan(b.kkt[0]));
    double* dth = malloc(sizeof(double) * B * P);
    int32_t* vs = malloc(sizeof(int32_t) * B);
    EXPECT(oracle_vjp_batch(&d, theta, b.x, b.y, b.s, b.x, b.y, NULL, dth, vs, 4) == 0);
    free(dth); free(vs);
    free_out(&b);
  }
  /* m = 0: no constraints */
  {
    mcpx_params p; params(&p, 1);
    bufs b; mcpx_out o = alloc_out(1, 2, 0, &b);
    const double t0[6] = {2, 0, 0, 2, 1, 1};
    mcpx_desc d = {MCPX_FAMILY_QP, 2, 0, 0, 1, 6};
    EXPECT(oracle_solve_batch(&d, t0, NULL, NULL, NULL, &p, &o, 1) == 0);
    EXPECT(b.status[0] == 0 && fabs(b.x[0] - 0.5) < 1e-9);
    free_out(&b);
  }
  free(theta);
  printf("oracle_checks: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
