// Streaming probe (timing tool, not product): in-place read-modify-write of one 2 GiB state
// (n = 28 f32, what a single-gate apply kernel does) against the same pattern out of place
// (read state A, write state B), with block-contiguous ranges of U 16-B items per thread in
// flight, with and without the XCD-aware block order the single-gate kernels use.  Prints
// TB/s (2S per launch) and the fraction of 8 TB/s, best of 5 after a warm-up.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/stream_probe tools/r5/stream_probe.hip
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
__device__ __forceinline__ vec4 ldp(const vec4* p) { return *p; }
__device__ __forceinline__ void stp(vec4* p, vec4 v) { *p = v; }

// block b owns items [b * 256 * U, (b + 1) * 256 * U); XCD: block b of G runs the range of
// (b % 8) * G / 8 + b / 8 (one contiguous eighth per XCD)
template <int U, bool XCD, bool NT>
__global__ __launch_bounds__(256) void k_stream(const vec4* __restrict__ a, vec4* __restrict__ b,
                                                uint64_t n) {
  uint64_t blk = blockIdx.x;
  if (XCD) blk = (uint64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const uint64_t i0 = blk * 256 * U + threadIdx.x;
  vec4 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) x[u] = NT ? ld(a + i0 + (uint64_t)u * 256) : ldp(a + i0 + (uint64_t)u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const vec4 y = x[u] * 0.9999999f + x[u].yxwz * 1e-7f;
    if (NT)
      st(b + i0 + (uint64_t)u * 256, y);
    else
      stp(b + i0 + (uint64_t)u * 256, y);
  }
}

// Gate-shaped patterns: ROWS rows (the 2^k amplitudes a k-qubit gate couples) at a far chunk
// stride (1 << RB).  SPLIT: one chunk per lane — lane group g = lane / (64 / ROWS) takes row g,
// so a wave covers 64 / ROWS consecutive items of each row; else each lane loads every row of
// its item (the single-gate direct kernels' shape: ROWS loads per lane).
template <int ROWS, bool SPLIT, int RB>
__global__ __launch_bounds__(256) void k_rows(vec4* __restrict__ a, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int LOGR = ROWS == 1 ? 0 : ROWS == 2 ? 1 : 2;
  auto row_addr = [&](uint64_t item, int r) {  // item: index over n / ROWS; insert row bits
    uint64_t x = item;
    for (int k = 0; k < LOGR; ++k) {
      const uint32_t b = RB + k;
      x = ((x >> b) << (b + 1)) | (x & ((1ull << b) - 1));
    }
    for (int k = 0; k < LOGR; ++k) x |= (uint64_t)((r >> k) & 1) << (RB + k);
    return x;
  };
  if (SPLIT) {
    const uint32_t per = 64 / ROWS, g = lane / per, i = lane % per;
    const uint64_t item = ((uint64_t)blockIdx.x * 4 + wave) * per + i;
    vec4 x = ld(a + row_addr(item, (int)g));
    x = x * 0.9999999f + x.yxwz * 1e-7f;
    st(a + row_addr(item, (int)g), x);
  } else {
    const uint64_t item = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    vec4 x[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) x[r] = ld(a + row_addr(item, r));
#pragma unroll
    for (int r = 0; r < ROWS; ++r) st(a + row_addr(item, r), x[r] * 0.9999999f + x[(r + 1) % ROWS] * 1e-7f);
  }
}

template <int ROWS, bool SPLIT, int RB>
static void run_rows(vec4* a, uint64_t n) {
  const uint32_t grid = SPLIT ? (uint32_t)(n / 256) : (uint32_t)(n / ROWS / 256);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_rows<ROWS, SPLIT, RB>), dim3(grid), dim3(256), 0, 0, a, n);
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_rows<ROWS, SPLIT, RB>), dim3(grid), dim3(256), 0, 0, a, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double tbs = 2.0 * (double)n * 16 / (best * 1e-3) / 1e12;
  printf("rows=%d split=%d rowbit=%2d             %7.3f ms  %5.2f TB/s  %5.1f%%\n", ROWS, SPLIT ? 1 : 0,
         RB, best, tbs, 100.0 * tbs / 8.0);
}

template <int U, bool XCD, bool NT>
static void run(const char* name, vec4* a, vec4* b, uint64_t n) {
  const uint32_t grid = (uint32_t)(n / (256 * U));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_stream<U, XCD, NT>), dim3(grid), dim3(256), 0, 0, a, b, n);
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_stream<U, XCD, NT>), dim3(grid), dim3(256), 0, 0, a, b, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double tbs = 2.0 * (double)n * 16 / (best * 1e-3) / 1e12;
  printf("%-28s U=%d xcd=%d nt=%d  %7.3f ms  %5.2f TB/s  %5.1f%%\n", name, U, XCD ? 1 : 0, NT ? 1 : 0,
         best, tbs, 100.0 * tbs / 8.0);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const uint64_t n = (1ull << 28) / 2;  // 16-B chunks of an f32 2^28 state
  vec4 *a, *b;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(b, 0, n * 16));
  for (int rep = 0; rep < 2; ++rep) {
    run<1, true, true>("in place", a, a, n);
    run<1, true, true>("out of place", a, b, n);
    run<2, true, true>("in place", a, a, n);
    run<2, true, true>("out of place", a, b, n);
    run<4, true, true>("in place", a, a, n);
    run<4, true, true>("out of place", a, b, n);
    run<1, false, true>("in place", a, a, n);
    run<1, false, true>("out of place", a, b, n);
    run<4, false, true>("in place", a, a, n);
    run<4, false, true>("out of place", a, b, n);
    run<1, true, false>("in place", a, a, n);
    run<1, true, false>("out of place", a, b, n);
  }
  for (int rep = 0; rep < 2; ++rep) {
    run_rows<2, false, 20>(a, n);
    run_rows<2, true, 20>(a, n);
    run_rows<2, false, 12>(a, n);
    run_rows<2, true, 12>(a, n);
    run_rows<4, false, 20>(a, n);
    run_rows<4, true, 20>(a, n);
    run_rows<4, false, 8>(a, n);
    run_rows<4, true, 8>(a, n);
  }
  return 0;
}
