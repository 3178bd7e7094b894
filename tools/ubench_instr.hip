// Lone-wave instruction costs on gfx950 (one wave per SIMD): cycles per instruction of
// independent / dependent FP64 fma, DPP row_newbcast fmac, readlane, readfirstlane.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/ubench_instr.hip -o tools/abx/ubench_instr
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T>
__global__ __launch_bounds__(64) void bench(double* out, unsigned long long* cyc, int reps) {
  const int ln = threadIdx.x;
  double a[16];
  for (int i = 0; i < 16; ++i) a[i] = ln * 0.001 + i;
  const double b = 1.0000001, c = 0.999999;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (T == 0) a[i] = __builtin_fma(a[i], b, c);  // 16 independent chains
        if (T == 1) a[0] = __builtin_fma(a[0], b, c);  // one dependent chain
        if (T == 2) asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(b));
        if (T == 3) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 15]), "v"(b));
        if (T == 4) {
          int lo = __builtin_amdgcn_readlane(__double2loint(a[i]), 5), hi = __builtin_amdgcn_readlane(__double2hiint(a[i]), 5);
          a[(i + 1) & 15] = __builtin_fma(__hiloint2double(hi, lo), b, a[(i + 1) & 15]);
        }
        if (T == 5) {
          unsigned x = __double2loint(a[i]);
          asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x) : "v"(x));
          a[i] = __hiloint2double(__double2hiint(a[i]), (int)x);
        }
        if (T == 6) a[i] = a[i] * b;  // v_mul_f64
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < 16; ++i) s += a[i];
  out[blockIdx.x * 64 + ln] = s;
  if (ln == 0) cyc[blockIdx.x] = (t1 - t0);
}

int main() {
  double* o;
  unsigned long long* c;
  hipMalloc(&o, 256 * 64 * 8);
  hipMalloc(&c, 256 * 8);
  const int reps = 200;
  const char* names[] = {"fma f64 independent", "fma f64 dependent chain", "v_fmac_f64_dpp row_newbcast",
                         "v_fmac_f64 (asm)", "readlane x2 + fma", "permlane16_swap (+mov)", "mul f64 independent"};
#define R(T)                                                                                  \
  {                                                                                           \
    hipLaunchKernelGGL(bench<T>, dim3(256), dim3(64), 0, 0, o, c, reps);                      \
    hipDeviceSynchronize();                                                                   \
    unsigned long long h[256];                                                                \
    hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost);                                         \
    double s = 0;                                                                             \
    for (int i = 0; i < 256; ++i) s += h[i];                                                  \
    printf("%-32s %6.2f cycles per (64-entry) op\n", names[T], s / 256 / (reps * 64.0));      \
  }
  R(0) R(1) R(2) R(3) R(4) R(5) R(6)
  return 0;
}
