// Streaming probe 3 (timing tool, not product): the fused passes' HBM pattern.  A persistent
// grid of one-wave blocks walks 2^10-chunk tiles (16 chunks per lane in flight, in place: read
// the tile, write it back), block-contiguous like the register-resident passes; a tile is 2^r
// contiguous chunks (rows of 16 * 2^r bytes) times 2^(10 - r) rows at far chunk bits
// (14, 15, ...).  By row length and waves per SIMD: what the apply pass's memory skeleton
// (128-B rows in two thirds of the C2 passes) can reach.  Also two-state (f and b) tiles.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/stream_probe3 tools/r5/stream_probe3.hip
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

// chunk offset of tile-local chunk c (10 bits): low r bits contiguous, row bits at 14..
__device__ __forceinline__ uint64_t local_off(uint32_t c, uint32_t r) {
  const uint64_t lo = c & ((1u << r) - 1u);
  const uint64_t row = c >> r;
  return lo | (row << 14);
}
// tile t's base: its bits fill chunk bits r..13 then 14 + (10 - r) .. upward
__device__ __forceinline__ uint64_t tile_base(uint64_t t, uint32_t r) {
  const uint32_t nlo = 14 - r;  // tile-index bits below the row bits
  const uint64_t lo = t & ((1ull << nlo) - 1ull);
  const uint64_t hi = t >> nlo;
  return (lo << r) | (hi << (14 + (10 - r)));
}

// ORDER 0: block-contiguous (tpb tiles per block); 1: grid-strided; 2: one global counter
// (tiles handed out in increasing order); 3: eight counters, XCD x takes its contiguous
// eighth in increasing order
template <bool TWO, int ORDER, int NL = 16>
__global__ __launch_bounds__(64) void k_tiles(vec4* __restrict__ f, vec4* __restrict__ b, uint64_t ntiles,
                                              uint32_t r, uint32_t tpb, unsigned long long* ctr) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * tpb;
  uint64_t off[NL];
#pragma unroll
  // NL = 16: the 2^10-chunk tile with rows (local_off); else a contiguous NL-KiB tile
  for (int i = 0; i < NL; ++i) off[i] = NL == 16 ? local_off((uint32_t)i * 64 + lane, r) : (uint64_t)i * 64 + lane;
  const uint32_t x = blockIdx.x & 7u;
  for (uint64_t s = 0;; ++s) {
    uint64_t t;
    if constexpr (ORDER == 4) {  // one tile per wave (a grid of ntiles one-wave blocks)
      if (s >= 1) break;
      t = blockIdx.x;
    } else if constexpr (ORDER == 0) {
      if (s >= tpb) break;
      t = t0 + s;
    } else if constexpr (ORDER == 1) {
      t = blockIdx.x + s * gridDim.x;
    } else {
      unsigned long long v = 0;
      if (lane == 0) v = atomicAdd(&ctr[ORDER == 2 ? 0 : x * 16], 1ull);
      v = __shfl(v, 0, 64);
      t = ORDER == 2 ? v : (uint64_t)x * (ntiles / 8) + v;
      if (ORDER == 3 && v >= ntiles / 8) break;
    }
    if (t >= ntiles) break;
    const uint64_t base = NL == 16 ? tile_base(t, r) : t * (64u * NL);
    vec4 x[NL], y[TWO ? NL : 1];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      x[i] = ld(f + base + off[i]);
      if constexpr (TWO) y[i] = ld(b + base + off[i]);
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      st(f + base + off[i], x[i] * 0.9999999f);
      if constexpr (TWO) st(b + base + off[i], y[i] * 0.9999999f);
    }
  }
}

static unsigned long long* g_ctr = nullptr;
template <bool TWO, int ORDER = 0, int NL = 16>
static void run(vec4* f, vec4* b, uint64_t nch, uint32_t r, uint32_t waves_per_simd) {
  const uint64_t ntiles = nch / (64u * NL);
  const uint32_t grid = ORDER == 4 ? (uint32_t)ntiles : 256u * 4u * waves_per_simd;
  const uint32_t tpb = (uint32_t)((ntiles + grid - 1) / grid);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(g_ctr, 0, 8 * 16 * 8));
  hipLaunchKernelGGL((k_tiles<TWO, ORDER, NL>), dim3(grid), dim3(64), 0, 0, f, b, ntiles, r, tpb, g_ctr);
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int k = 0; k < 5; ++k) {
    CK(hipMemset(g_ctr, 0, 8 * 16 * 8));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_tiles<TWO, ORDER, NL>), dim3(grid), dim3(64), 0, 0, f, b, ntiles, r, tpb, g_ctr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double bytes = (TWO ? 4.0 : 2.0) * (double)nch * 16;
  const double tbs = bytes / (best * 1e-3) / 1e12;
  printf("%s order %d tile %5u B rows of %5u B  waves/SIMD %u  %7.3f ms  %5.2f TB/s  %5.1f%%\n",
         TWO ? "two-state" : "one-state", ORDER, 1024u * NL, NL == 16 ? 16u << r : 1024u * NL, waves_per_simd,
         best, tbs, 100.0 * tbs / 8.0);
  fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const uint64_t nch = (1ull << 28) / 2;  // f32 2^28 state in 16-B chunks
  vec4 *f, *b;
  CK(hipMalloc(&f, nch * 16));
  CK(hipMalloc(&b, nch * 16));
  CK(hipMemset(f, 0, nch * 16));
  CK(hipMemset(b, 0, nch * 16));
  CK(hipMalloc(&g_ctr, 8 * 16 * 8));
  // one tile per wave (non-persistent) against the persistent block-contiguous walk
  for (uint32_t r : {3u, 10u}) {
    run<false, 4, 16>(f, b, nch, r, 1);
    run<false, 0, 16>(f, b, nch, r, 2);
    run<true, 4, 16>(f, b, nch, r, 1);
    run<true, 0, 16>(f, b, nch, r, 2);
  }
  run<false, 4, 1>(f, b, nch, 0, 1);
  run<false, 4, 4>(f, b, nch, 0, 1);
  run<false, 4, 8>(f, b, nch, 0, 1);
  run<true, 4, 4>(f, b, nch, 0, 1);
  run<true, 4, 8>(f, b, nch, 0, 1);
  return 0;
}
