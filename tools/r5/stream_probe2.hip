// Streaming probe 2 (timing tool, not product): where gate-shaped in-place passes over one
// 2 GiB state (n = 28 f32) lose HBM bandwidth.
//   rows:   an R-row gate pattern (rows at chunk bits rb0 [, rb1]), one chunk per lane, lane
//           groups per row (a wave covers 64 / R consecutive items of each row), by row bit;
//   lds:    the same pattern with whole waves per row: a block of NT threads loads NT / R
//           consecutive chunks of each row and exchanges through LDS (each wave instruction
//           moves one contiguous KiB);
//   two:    two-state in-place elementwise (f and b read and written: the reverse sweep's
//           per-gate kernels) with a block-reduction epilogue, by grid size and items in flight.
// Prints TB/s (algorithmic bytes per launch) and the fraction of 8 TB/s, best of 5 after a warm-up.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/stream_probe2 tools/r5/stream_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float vec4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) vec4 gvec4;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ vec4 ld(const vec4* p) { return __builtin_nontemporal_load((const gvec4*)p); }
__device__ __forceinline__ void st(vec4* p, vec4 v) { __builtin_nontemporal_store(v, (gvec4*)p); }

__device__ __forceinline__ uint64_t ins0(uint64_t x, uint32_t b) {
  const uint64_t low = x & ((1ull << b) - 1ull);
  return ((x - low) << 1) | low;
}
__device__ __forceinline__ uint32_t xcd(uint32_t b, uint32_t g) {
  return (g & 7u) ? b : (b & 7u) * (g >> 3) + (b >> 3);
}

// lane-group rows: lane l takes row l / (64 / R) of item (wave * 64 / R + l % (64 / R))
template <int R>
__global__ __launch_bounds__(256) void k_rows(vec4* __restrict__ a, uint32_t rb0, uint32_t rb1) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t PER = 64 / R;
  const uint32_t g = lane / PER;
  const uint64_t item = ((uint64_t)xcd(blockIdx.x, gridDim.x) * 4 + wave) * PER + lane % PER;
  uint64_t c = ins0(item, rb0);
  if (R == 4) c = ins0(c, rb1);
  c |= (uint64_t)(g & 1) << rb0;
  if (R == 4) c |= (uint64_t)(g >> 1) << rb1;
  vec4 x = ld(a + c);
  x = x * 0.9999999f + x.yxwz * 1e-7f;
  st(a + c, x);
}

// whole waves per row, exchange through LDS: NT threads = R groups of NT / R consecutive chunks
template <int R, int NT>
__global__ __launch_bounds__(NT) void k_lds(vec4* __restrict__ a, uint32_t rb0, uint32_t rb1) {
  __shared__ vec4 s[NT];
  constexpr uint32_t PER = NT / R;
  const uint32_t t = threadIdx.x, g = t / PER;
  const uint64_t item = (uint64_t)xcd(blockIdx.x, gridDim.x) * PER + t % PER;
  uint64_t c = ins0(item, rb0);
  if (R == 4) c = ins0(c, rb1);
  c |= (uint64_t)(g & 1) << rb0;
  if (R == 4) c |= (uint64_t)(g >> 1) << rb1;
  vec4 x = ld(a + c);
  s[t] = x;
  __syncthreads();
  vec4 y = x * 0.9999999f;
#pragma unroll
  for (int r = 1; r < R; ++r) y += s[(t + r * PER) % NT] * 1e-7f;
  st(a + c, y);
}

// two-state in-place elementwise with U items in flight and `it` items per thread, plus a
// block reduction of one float (the per-gate reverse kernels' shape)
template <int U>
__global__ __launch_bounds__(256) void k_two(vec4* __restrict__ f, vec4* __restrict__ b, uint32_t it,
                                             float* __restrict__ part) {
  __shared__ float red[4];
  const uint64_t start = (uint64_t)blockIdx.x * 256 * it + threadIdx.x;
  float acc = 0;
  for (uint32_t s = 0; s < it; s += U) {
    vec4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = ld(f + start + (uint64_t)(s + u) * 256);
      y[u] = ld(b + start + (uint64_t)(s + u) * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc += x[u].x * y[u].y;
      st(f + start + (uint64_t)(s + u) * 256, x[u] * 0.9999999f);
      st(b + start + (uint64_t)(s + u) * 256, y[u] * 0.9999999f);
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

template <typename F>
static float best_of(F launch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  launch();
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return best;
}

static void report(const char* what, float ms, double bytes) {
  const double tbs = bytes / (ms * 1e-3) / 1e12;
  printf("%-44s %7.3f ms  %5.2f TB/s  %5.1f%%\n", what, ms, tbs, 100.0 * tbs / 8.0);
  fflush(stdout);
}

int main() {
  const uint64_t n = (1ull << 28) / 2;  // 16-B chunks of an f32 2^28 state
  vec4 *a, *b;
  float* part;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&part, 1 << 22));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(b, 0, n * 16));
  char what[96];
  const double S2 = 2.0 * (double)n * 16;
  const uint32_t bits[] = {6, 8, 10, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26};
  for (uint32_t rb : bits) {
    float ms = best_of([&] { hipLaunchKernelGGL(k_rows<2>, dim3(n / 256), dim3(256), 0, 0, a, rb, 0u); });
    snprintf(what, sizeof what, "rows R=2 rb=%u", rb);
    report(what, ms, S2);
  }
  for (uint32_t rb : bits) {
    if (rb == 6) continue;
    const uint32_t lo = rb == 8 ? 6 : 8;
    float ms = best_of([&] { hipLaunchKernelGGL(k_rows<4>, dim3(n / 256), dim3(256), 0, 0, a, lo, rb); });
    snprintf(what, sizeof what, "rows R=4 rb=%u,%u", lo, rb);
    report(what, ms, S2);
    if (rb >= 10) {
      ms = best_of([&] { hipLaunchKernelGGL(k_rows<4>, dim3(n / 256), dim3(256), 0, 0, a, rb - 1, rb); });
      snprintf(what, sizeof what, "rows R=4 rb=%u,%u", rb - 1, rb);
      report(what, ms, S2);
    }
  }
  for (uint32_t rb : {12u, 16u, 20u, 24u, 26u}) {
    float ms = best_of([&] { hipLaunchKernelGGL((k_lds<2, 256>), dim3(n / 256), dim3(256), 0, 0, a, rb, 0u); });
    snprintf(what, sizeof what, "lds R=2 NT=256 rb=%u", rb);
    report(what, ms, S2);
    ms = best_of([&] { hipLaunchKernelGGL((k_lds<2, 1024>), dim3(n / 1024), dim3(1024), 0, 0, a, rb, 0u); });
    snprintf(what, sizeof what, "lds R=2 NT=1024 rb=%u", rb);
    report(what, ms, S2);
    ms = best_of([&] { hipLaunchKernelGGL((k_lds<4, 256>), dim3(n / 256), dim3(256), 0, 0, a, rb - 1, rb); });
    snprintf(what, sizeof what, "lds R=4 NT=256 rb=%u,%u", rb - 1, rb);
    report(what, ms, S2);
    ms = best_of([&] { hipLaunchKernelGGL((k_lds<4, 1024>), dim3(n / 1024), dim3(1024), 0, 0, a, rb - 1, rb); });
    snprintf(what, sizeof what, "lds R=4 NT=1024 rb=%u,%u", rb - 1, rb);
    report(what, ms, S2);
  }
  const double S4 = 2.0 * S2;
  for (uint32_t grid : {2048u, 4096u, 8192u, 16384u, 65536u, 524288u}) {
    const uint32_t it = (uint32_t)(n / 256 / grid);
    float ms = best_of([&] { hipLaunchKernelGGL(k_two<1>, dim3(grid), dim3(256), 0, 0, a, b, it, part); });
    snprintf(what, sizeof what, "two U=1 grid=%u it=%u", grid, it);
    report(what, ms, S4);
    if (it >= 2) {
      ms = best_of([&] { hipLaunchKernelGGL(k_two<2>, dim3(grid), dim3(256), 0, 0, a, b, it, part); });
      snprintf(what, sizeof what, "two U=2 grid=%u it=%u", grid, it);
      report(what, ms, S4);
    }
    if (it >= 4) {
      ms = best_of([&] { hipLaunchKernelGGL(k_two<4>, dim3(grid), dim3(256), 0, 0, a, b, it, part); });
      snprintf(what, sizeof what, "two U=4 grid=%u it=%u", grid, it);
      report(what, ms, S4);
    }
  }
  return 0;
}
