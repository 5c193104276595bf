// Prints the operand/result lane layout of v_mfma_f32_4x4x1_16b_f32 (one instruction from zero):
// checks D(lane l, reg r) == a(lane 4*(l/4) + r) * b(lane l), i.e. block = l/4, row i = r, col j = l%4.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/mfma_layout_probe tools/mfma_layout_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out) {
  const int l = threadIdx.x;
  const float a = 1.0f + l, b = 1000.0f + l;
  f4 d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
}
int main() {
  float* o;
  (void)hipMalloc(&o, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
  float h[256];
  (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const float want = (1.0f + 4 * (l / 4) + r) * (1000.0f + l);
      if (h[l * 4 + r] != want) ++bad;
    }
  printf("layout block=l/4,i=r,j=l%%4: %s (%d mismatches)\n", bad ? "NO" : "YES", bad);
  for (int l = 0; l < 8; ++l)
    printf("lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
