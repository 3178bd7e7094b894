// Micro-benchmarks for the LU elimination inner step on gfx950:
//   a_j ← fma(−l, u_j, a_j) for j = 0..NJ-1, u_j = pivot row broadcast from lane p.
// Variants of the broadcast: readlane→SGPR, LDS (pivot lane writes, all read),
// ds_bpermute, and a no-broadcast FMA-only reference.  Prints ns and cycles
// per element-update per wave for several waves-per-SIMD counts.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_bcast.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define NJ 32
#define REPS 256

__device__ __forceinline__ double rl(double v, int src) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ __launch_bounds__(64) void k(double* out, double l0, int seed) {
  __shared__ __attribute__((aligned(16))) double row[NJ];
  const int lane = threadIdx.x;
  double a[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) a[j] = 1.0 + 1e-3 * (lane + j);
  double l = l0 * (1 + lane * 1e-6);
  for (int r = 0; r < REPS; ++r) {
    const int p = (r * 7 + seed) & 63;
    if (MODE == 0) {  // FMA only, uniform SGPR operand (no broadcast)
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = fma(-l, l0, a[j]);
    } else if (MODE == 1) {  // readlane broadcast
#pragma unroll
      for (int j = 0; j < NJ; ++j) a[j] = fma(-l, rl(a[j], p), a[j]);
    } else if (MODE == 2) {  // LDS: pivot lane writes row, all lanes read
      if (lane == p) {
#pragma unroll
        for (int j = 0; j < NJ; j += 2) *(double2*)&row[j] = make_double2(a[j], a[j + 1]);
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < NJ; j += 2) {
        const double2 u = *(const double2*)&row[j];
        a[j] = fma(-l, u.x, a[j]);
        a[j + 1] = fma(-l, u.y, a[j + 1]);
      }
      __syncthreads();
    } else if (MODE == 3) {  // ds_bpermute broadcast
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int lo = __builtin_amdgcn_ds_bpermute(p * 4, __double2loint(a[j]));
        int hi = __builtin_amdgcn_ds_bpermute(p * 4, __double2hiint(a[j]));
        a[j] = fma(-l, __hiloint2double(hi, lo), a[j]);
      }
    } else if (MODE == 4) {  // readlane only (consumed by an add into one acc)
      double acc = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc += rl(a[j], p);
      a[r & (NJ - 1)] += acc * 1e-30;
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += a[j];
  out[blockIdx.x * 64 + lane] = s;
}

template <int MODE>
float run(int blocks, double* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, d, 0.5, 3);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, d, 0.5, 3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* d;
  hipMalloc(&d, sizeof(double) * 64 * 256 * 64);
  const char* names[] = {"fma-only(sgpr)", "readlane+fma", "lds-bcast+fma", "bpermute+fma", "readlane-only"};
  for (int wps : {1, 2, 3, 4, 8}) {
    const int blocks = 256 * 4 * wps;  // waves = blocks, per SIMD = wps
    float t[5] = {run<0>(blocks, d), run<1>(blocks, d), run<2>(blocks, d), run<3>(blocks, d), run<4>(blocks, d)};
    for (int mde = 0; mde < 5; ++mde) {
      // element-updates per SIMD = wps * REPS * NJ ; cycles at 2.4 GHz nominal
      const double per = (double)wps * REPS * NJ;
      printf("waves/SIMD=%d %-16s %8.3f ms  %6.2f ns/update/SIMD  %6.2f cyc@2.4GHz\n", wps, names[mde], t[mde],
             t[mde] * 1e6 / per, t[mde] * 1e6 / per * 2.4);
    }
  }
  return 0;
}
