// Prints the lane layout of v_mfma_f64_16x16x4f64: for A one-hot in lane L (B lane l = l + 1),
// the nonzero D entries (lane, register, value) — value = the B lane + 1 that pairs with L.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/mfma_f64_layout_probe tools/mfma_f64_layout_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out, int L) {
  const int l = threadIdx.x;
  const double a = l == L ? 1.0 : 0.0, b = 1.0 + l;
  d4 d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
}
int main() {
  double* o;
  (void)hipMalloc(&o, 256 * 8);
  for (int L : {0, 1, 2, 15, 16, 17, 32, 48}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, L);
    double h[256];
    (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
    printf("A one-hot lane %2d:", L);
    int cnt = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r)
        if (h[l * 4 + r] != 0 && cnt++ < 20) printf(" (%d,%d)=%g", l, r, h[l * 4 + r] - 1);
    printf("  [%d nonzero]\n", cnt);
  }
  return 0;
}
