// VALU throughput probe (gfx950): FMA rate of the instruction forms the fused kernels use.
//   pk_s_opsel : v_pk_fma_f32 with a uniform SGPR-pair operand + op_sel/neg modifiers (ucfma)
//   pk_v       : v_pk_fma_f32 with VGPR operands, no modifiers
//   fma        : v_fma_f32
// Each thread runs CH independent accumulator chains for ITER steps; rate = FMAs / time.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int CH = 8;
constexpr int ITER = 4096;

__global__ void k_pk_s(f2* out, f2 m0, f2 m1) {
  f2 acc[CH];
  f2 x = {(float)threadIdx.x, 1.0f};
  for (int c = 0; c < CH; ++c) acc[c] = {0.f, (float)c};
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[c]) : "s"(m0), "v"(x));
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
                   : "+v"(acc[c]) : "s"(m1), "v"(x));
    }
  }
  f2 s = acc[0];
  for (int c = 1; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pk_v(f2* out, float a) {
  f2 acc[CH];
  f2 x = {(float)threadIdx.x, 1.0f};
  f2 m = {a, a + 1.0f};
  for (int c = 0; c < CH; ++c) acc[c] = {0.f, (float)c};
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(m), "v"(x));
#pragma unroll
    for (int c = 0; c < CH; ++c)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(m), "v"(x));
  }
  f2 s = acc[0];
  for (int c = 1; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma(f2* out, float a) {
  float acc[2 * CH];
  float x = (float)threadIdx.x;
  for (int c = 0; c < 2 * CH; ++c) acc[c] = (float)c;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < 2 * CH; ++c)
      asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(x));
#pragma unroll
    for (int c = 0; c < 2 * CH; ++c)
      asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(x));
  }
  float s = 0;
  for (int c = 0; c < 2 * CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = f2{s, s};
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int block = 256;
  f2* out;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int wpsimd : {1, 2, 4, 8}) {
    const int grid = cus * wpsimd;  // 4 waves per block = one per SIMD
    hipMalloc(&out, sizeof(f2) * grid * block);
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        if (kind == 0) hipLaunchKernelGGL(k_pk_s, dim3(grid), dim3(block), 0, 0, out, f2{1.0f, 0.5f}, f2{0.25f, 0.125f});
        if (kind == 1) hipLaunchKernelGGL(k_pk_v, dim3(grid), dim3(block), 0, 0, out, 1.0f);
        if (kind == 2) hipLaunchKernelGGL(k_fma, dim3(grid), dim3(block), 0, 0, out, 1.0f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      // FMAs: per thread ITER * 2*CH instructions, packed = 2 FMAs each
      const double instr = (double)grid * block * ITER * 2 * CH * (kind == 2 ? 2 : 1);
      const double fmas = instr * (kind == 2 ? 1 : 2);
      const double tflops = 2 * fmas / (best * 1e-3) / 1e12;
      // cycles per wave-instruction per SIMD at 2.4 GHz
      const double wave_instr_per_simd = instr / 64.0 / (cus * 4.0);
      const double cyc = best * 1e-3 * 2.4e9 / wave_instr_per_simd;
      printf("waves/SIMD %d  %-10s  %.3f ms  %.1f TFLOP/s  %.2f cycles/wave-instr (@2.4GHz)\n", wpsimd,
             kind == 0 ? "pk_s_opsel" : kind == 1 ? "pk_v" : "fma", best, tflops, cyc);
    }
    hipFree(out);
  }
  return 0;
}
