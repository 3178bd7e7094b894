// Semantics check of the cross-lane primitives the 2-D Gauss-Jordan relies on
// (gfx950): v_permlane16_swap / v_permlane32_swap and DPP row_newbcast on f64.
// Prints OK/FAIL per primitive.  Build: hipcc --offload-arch=gfx950 -O2 tools/ubench_lanes.hip -o tools/ubench_lanes
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out, double* dout) {
  const unsigned l = threadIdx.x;
  const unsigned x = 1000 + l;
  auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  auto p32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  out[0 * 64 + l] = p16[0];
  out[1 * 64 + l] = p16[1];
  out[2 * 64 + l] = p32[0];
  out[3 * 64 + l] = p32[1];
  const double v = 0.5 + l;
  dout[l] = __builtin_amdgcn_update_dpp(0.0, v, 0x153, 0xf, 0xf, false);  // row_newbcast:3
  double r;
  asm volatile("v_mov_b64 %0, 0\n s_nop 1\n v_fmac_f64_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf"
               : "=&v"(r) : "v"(v), "v"(2.0));
  dout[64 + l] = r;
}

int main() {
  unsigned* o; double* d;
  (void)hipMalloc(&o, 4 * 64 * 4); (void)hipMalloc(&d, 128 * 8);
  k<<<1, 64>>>(o, d);
  unsigned h[256]; double hd[128];
  (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hd, d, sizeof hd, hipMemcpyDeviceToHost);
  for (int t = 0; t < 4; ++t) {
    printf("out%d:", t);
    for (int row = 0; row < 4; ++row) printf(" row%d<-lane %u..%u", row, h[t * 64 + 16 * row] - 1000, h[t * 64 + 16 * row + 15] - 1000);
    printf("\n");
  }
  int ok = 1;
  for (int l = 0; l < 64; ++l) ok &= hd[l] == 0.5 + (l / 16) * 16 + 3;
  printf("update_dpp f64 row_newbcast:3 %s\n", ok ? "OK" : "FAIL");
  ok = 1;
  for (int l = 0; l < 64; ++l) ok &= hd[64 + l] == (0.5 + (l / 16) * 16 + 5) * 2.0;
  printf("v_fmac_f64_dpp row_newbcast:5 %s\n", ok ? "OK" : "FAIL");
  return 0;
}
