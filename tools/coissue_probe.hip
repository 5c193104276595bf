// Co-issue probe (gfx950): do f32 MFMA waves and f32 VALU waves share a SIMD without slowing
// each other?  One 512-thread block per CU = 2 waves per SIMD.  Modes:
//   role 0: every wave runs the MFMA stream only
//   role 1: every wave runs the VALU stream only
//   role 2: waves 0-3 (one per SIMD) MFMA, waves 4-7 VALU (separate waves, same SIMD)
//   role 3: every wave runs both streams interleaved
// MFMA forms: 4x4x1_16b f32 (M=0) or 16x16x4 f32 (M=1).  VALU forms: v_pk_fma_f32 (V=0) or
// v_fma_f32 (V=1).  Prints ms and cycles per iteration per wave.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/coissue_probe tools/coissue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;

template <int M>
__device__ __forceinline__ void mfma_step(f4 (&c)[4], float a, float b) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (M == 0) c[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[i], 0, 0, 0);
    else c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
  }
}
template <int V, int NV>
__device__ __forceinline__ void valu_step(f2 (&v)[8], f2 m) {
#pragma unroll
  for (int r = 0; r < NV / 8; ++r)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if constexpr (V == 0)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(v[c]) : "v"(m), "v"(v[(c + 1) & 7]));
      else
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[c].x) : "v"(m.x), "v"(v[(c + 1) & 7].y));
    }
}

template <int ROLE, int M, int V, int NV>
__global__ __launch_bounds__(512) void k_probe(float* out, float a0) {
  f4 c[4] = {};
  f2 v[8];
  for (int i = 0; i < 8; ++i) v[i] = {(float)i, 1.0f};
  const float a = a0 + threadIdx.x * 1e-7f, b = a0 * 0.5f;
  const f2 m = {a, b};
  const int wave = threadIdx.x >> 6;
  const bool do_m = ROLE == 0 || ROLE == 3 || (ROLE == 2 && wave < 4);
  const bool do_v = ROLE == 1 || ROLE == 3 || (ROLE == 2 && wave >= 4);
  if (do_m && do_v) {
    for (int it = 0; it < ITER; ++it) {
      mfma_step<M>(c, a, b);
      valu_step<V, NV>(v, m);
    }
  } else if (do_m) {
    for (int it = 0; it < ITER; ++it) mfma_step<M>(c, a, b);
  } else {
    for (int it = 0; it < ITER; ++it) valu_step<V, NV>(v, m);
  }
  f4 s = c[0] + c[1] + c[2] + c[3];
  f2 t = v[0] + v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w + t.x + t.y;
}

template <int ROLE, int M, int V, int NV>
void run(const char* name, int cus, float* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_probe<ROLE, M, V, NV>), dim3(cus), dim3(512), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  printf("%-44s %.3f ms  %6.1f cyc/iter (per SIMD, 2.4 GHz)\n", name, best,
         best * 1e-3 * 2.4e9 / ITER);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  (void)hipMalloc(&out, sizeof(float) * cus * 512);
  run<0, 0, 0, 16>("4x4x1 x4, 2 waves/SIMD", cus, out);
  run<0, 1, 0, 16>("16x16x4 x4, 2 waves/SIMD", cus, out);
  run<1, 0, 0, 16>("pk_fma x16, 2 waves/SIMD", cus, out);
  run<1, 0, 1, 32>("fma x32, 2 waves/SIMD", cus, out);
  run<2, 0, 0, 16>("split: 4x4x1 x4 | pk_fma x16", cus, out);
  run<2, 0, 1, 32>("split: 4x4x1 x4 | fma x32", cus, out);
  run<2, 1, 0, 16>("split: 16x16x4 x4 | pk_fma x16", cus, out);
  run<2, 1, 1, 32>("split: 16x16x4 x4 | fma x32", cus, out);
  run<3, 0, 0, 16>("mixed: 4x4x1 x4 + pk_fma x16", cus, out);
  run<3, 0, 1, 32>("mixed: 4x4x1 x4 + fma x32", cus, out);
  run<3, 1, 0, 16>("mixed: 16x16x4 x4 + pk_fma x16", cus, out);
  run<3, 1, 1, 32>("mixed: 16x16x4 x4 + fma x32", cus, out);
  (void)hipFree(out);
  return 0;
}
