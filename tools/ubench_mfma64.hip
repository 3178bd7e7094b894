// (1) Numerics of v_mfma_f64_16x16x4_f64 on gfx950: is D = C + A·B an ordered
//     fma chain over k (bit-identical to fma(a3,b3,fma(a2,b2,fma(a1,b1,fma(a0,b0,c)))))?
// (2) Throughput of readlane variants (clustered vs interleaved, constant vs SGPR lane).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma64.hip -o tools/ubench_mfma64
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void mfma_test(const double* A, const double* B, const double* Cm, double* D, int trials) {
  const int l = threadIdx.x;
  for (int t = 0; t < trials; ++t) {
    const double* a = A + t * 64;
    const double* b = B + t * 64;
    const double* c = Cm + t * 256;
    double av = a[(l & 15) * 4 + (l >> 4)];  // A[i=l&15][k=l>>4], A stored row-major 16x4
    double bv = b[(l >> 4) * 16 + (l & 15)]; // B[k=l>>4][j=l&15], B stored row-major 4x16
    d4 cv;
    for (int r = 0; r < 4; ++r) cv[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
    d4 dv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, cv, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[t * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = dv[r];
  }
}

__device__ __forceinline__ double rl(double v, int src) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

#define NJ 32
#define REPS 256
template <int MODE>
__global__ __launch_bounds__(64) void rlk(double* out, double l0, int seed) {
  const int lane = threadIdx.x;
  double a[NJ];
  float f[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) { a[j] = 1.0 + 1e-3 * (lane + j); f[j] = (float)a[j]; }
  double l = l0 * (1 + lane * 1e-6);
  float lf = (float)l;
  for (int r = 0; r < REPS; ++r) {
    const int p = (r * 7 + seed) & 63;
    if (MODE == 0) {  // interleaved, SGPR lane
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = fma(-l, rl(a[j], p), a[j]);
    } else if (MODE == 1) {  // clusters of 8 readlane pairs then 8 fma
#pragma unroll
      for (int j0 = 0; j0 < NJ; j0 += 8) {
        double u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = rl(a[j0 + j], p);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j0 + j] = fma(-l, u[j], a[j0 + j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (MODE == 2) {  // constant lane
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = fma(-l, rl(a[j], 5), a[j]);
    } else if (MODE == 3) {  // f32: one readlane per element
#pragma unroll
      for (int j = 0; j < NJ; ++j) f[j] = fmaf(-lf, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f[j]), p)), f[j]);
    } else if (MODE == 4) {  // readfirstlane after moving pivot to lane 0 is not possible; test v_readfirstlane cost
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int lo = __builtin_amdgcn_readfirstlane(__double2loint(a[j]));
        int hi = __builtin_amdgcn_readfirstlane(__double2hiint(a[j]));
        a[j] = fma(-l, __hiloint2double(hi, lo), a[j]);
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += a[j] + f[j];
  out[blockIdx.x * 64 + lane] = s;
}

template <int MODE>
float run(int blocks, double* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rlk<MODE>, dim3(blocks), dim3(64), 0, 0, d, 0.5, 3);
  (void)hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(rlk<MODE>, dim3(blocks), dim3(64), 0, 0, d, 0.5, 3);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int T = 2000;
  std::mt19937_64 g(42);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::vector<double> A(T * 64), B(T * 64), C(T * 256), D(T * 256);
  for (auto& v : A) v = nd(g) * std::exp2((int)(g() % 20) - 10);
  for (auto& v : B) v = nd(g) * std::exp2((int)(g() % 20) - 10);
  for (auto& v : C) v = nd(g) * std::exp2((int)(g() % 20) - 10);
  double *dA, *dB, *dC, *dD;
  (void)hipMalloc(&dA, A.size() * 8); (void)hipMalloc(&dB, B.size() * 8);
  (void)hipMalloc(&dC, C.size() * 8); (void)hipMalloc(&dD, D.size() * 8);
  (void)hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_test, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, T);
  (void)hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
  long eq_chain = 0, eq_rev = 0, eq_exact = 0, eq_pair = 0, total = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const double* a = &A[t * 64 + i * 4];
        double bk[4];
        for (int k = 0; k < 4; ++k) bk[k] = B[t * 64 + k * 16 + j];
        const double c = C[t * 256 + i * 16 + j];
        double ch = c;
        for (int k = 0; k < 4; ++k) ch = std::fma(a[k], bk[k], ch);
        double rv = c;
        for (int k = 3; k >= 0; --k) rv = std::fma(a[k], bk[k], rv);
        long double ex = (long double)c;
        for (int k = 0; k < 4; ++k) ex += (long double)a[k] * (long double)bk[k];
        double pr = c + ((a[0] * bk[0] + a[1] * bk[1]) + (a[2] * bk[2] + a[3] * bk[3]));
        const double d = D[t * 256 + i * 16 + j];
        eq_chain += (d == ch);
        eq_rev += (d == rv);
        eq_exact += (d == (double)ex);
        eq_pair += (d == pr);
        ++total;
      }
  printf("mfma_f64_16x16x4: total %ld  ==fma-chain(k asc) %ld  ==fma-chain(k desc) %ld  ==round(longdouble) %ld  ==pairwise %ld\n",
         total, eq_chain, eq_rev, eq_exact, eq_pair);
  double* d;
  (void)hipMalloc(&d, sizeof(double) * 64 * 256 * 64);
  const char* names[] = {"interleaved/sgpr-lane", "clustered8/sgpr-lane", "interleaved/const-lane", "f32 readlane+fmaf",
                         "readfirstlane+fma"};
  for (int wps : {1, 2, 4}) {
    const int blocks = 256 * 4 * wps;
    float t[5] = {run<0>(blocks, d), run<1>(blocks, d), run<2>(blocks, d), run<3>(blocks, d), run<4>(blocks, d)};
    for (int md = 0; md < 5; ++md) {
      const double per = (double)wps * REPS * NJ;
      printf("waves/SIMD=%d %-24s %6.2f cyc/update@2.4GHz\n", wps, names[md], t[md] * 1e6 / per * 2.4);
    }
  }
  return 0;
}
