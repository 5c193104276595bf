// MFMA probe (gfx950): issue cost of the small f32 MFMA forms and whether VALU packed FMAs
// co-issue with them (same wave stream, independent registers).
//   mfma4     : v_mfma_f32_4x4x1_16b_f32, 4 independent accumulators
//   mfma16    : v_mfma_f32_16x16x4_f32, 4 independent accumulators
//   valu      : v_pk_fma_f32, 8 independent chains (the fused kernels' instruction form)
//   mix       : mfma4 + valu interleaved 1:R in one wave
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;

template <int KIND, int R>
__global__ void k_probe(float* out, float a0) {
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f2 v[8];
  for (int i = 0; i < 8; ++i) v[i] = {(float)i, 1.0f};
  const float a = a0 + threadIdx.x * 1e-7f, b = a0 * 0.5f;
  const f2 m = {a, b};
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0 || KIND == 3) {
      c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, b, c3, 0, 0, 0);
    }
    if constexpr (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
    }
    if constexpr (KIND == 2 || KIND == 3) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c)
          asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(v[c]) : "v"(m), "v"(v[(c + 1) & 7]));
    }
  }
  f4 s = c0 + c1 + c2 + c3;
  f2 t = v[0] + v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w + t.x + t.y;
}

template <int KIND, int R>
void run(const char* name, int cus, float* out, int mfma_per_iter, int valu_per_iter) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = cus * 4;  // one wave per SIMD per block of 64... 4 blocks of 64 per CU
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_probe<KIND, R>), dim3(grid), dim3(64), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  // one wave per SIMD: cycles per iteration at the measured time (2.4 GHz nominal)
  const double cyc_iter = best * 1e-3 * 2.4e9 / ITER;
  printf("%-22s %.3f ms  %.1f cycles/iter  (%d mfma + %d valu per iter)\n", name, best, cyc_iter,
         mfma_per_iter, valu_per_iter);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * cus * 4 * 64);
  run<0, 1>("mfma 4x4x1_16b", cus, out, 4, 0);
  run<1, 1>("mfma 16x16x4", cus, out, 4, 0);
  run<2, 1>("valu pk_fma x8", cus, out, 0, 8);
  run<2, 2>("valu pk_fma x16", cus, out, 0, 16);
  run<3, 1>("mix 4 mfma4 + 8 pk", cus, out, 4, 8);
  run<3, 2>("mix 4 mfma4 + 16 pk", cus, out, 4, 16);
  run<3, 4>("mix 4 mfma4 + 32 pk", cus, out, 4, 32);
  (void)hipFree(out);
  return 0;
}
