// Placement probe (timing tool, not product).  bench.py --micro shows the single-gate reverse
// kernels alternating between 63-65 % and 79 % of 8 TB/s from one fresh circuit to the next:
// the rate of a two-state in-place stream depends on where its two 2 GiB states were placed.
// Each trial here allocates states the way a circuit does (initial, state; bwd at the first
// backward), runs the two-state in-place stream (the k_diag / k_direct shape: one 16-B chunk
// per state per thread, a block per 256 chunks) on every pair, prints the virtual addresses and
// rates, and frees everything.  Then: one allocation holding both states, bwd at several
// offsets from fwd.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/alloc_probe tools/alloc_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

// pair kernel: item j covers chunks c0 = insert_zero(j, lb) and c0 + 2^lb of both states (the
// k_direct q1 row pattern at chunk bit lb)
__global__ __launch_bounds__(256) void k_pair(vec4* __restrict__ f, vec4* __restrict__ b, uint32_t lb) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t lo = j & ((1ull << lb) - 1);
  const uint64_t c0 = ((j - lo) << 1) | lo, c1 = c0 + (1ull << lb);
  vec4 x0 = ld(f + c0), x1 = ld(f + c1), y0 = ld(b + c0), y1 = ld(b + c1);
  st(f + c0, x0 * 1.0000001f);
  st(f + c1, x1 * 1.0000001f);
  st(b + c0, y0 * 0.9999999f);
  st(b + c1, y1 * 0.9999999f);
}

// quad kernel: item j covers chunks c0 + {0, 2^lb, 2^lb2, 2^lb + 2^lb2} of both states, lb < lb2
// (a q1 row pair at chunk bit lb, split over a second "bank" bit lb2)
__global__ __launch_bounds__(256) void k_quad(vec4* __restrict__ f, vec4* __restrict__ b, uint32_t lb,
                                              uint32_t lb2) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t lo = j & ((1ull << lb) - 1);
  uint64_t c0 = ((j - lo) << 1) | lo;
  lo = c0 & ((1ull << lb2) - 1);
  c0 = ((c0 - lo) << 1) | lo;
  const uint64_t o[4] = {0, 1ull << lb, 1ull << lb2, (1ull << lb) + (1ull << lb2)};
  vec4 x[4], y[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[k] = ld(f + c0 + o[k]);
    y[k] = ld(b + c0 + o[k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    st(f + c0 + o[k], x[k] * 1.0000001f);
    st(b + c0 + o[k], y[k] * 0.9999999f);
  }
}

// interleaved two-state buffer: state s, chunk j lives at insert_zero(j, g) + s * 2^g (fwd and
// bwd alternate in 2^g-chunk blocks of one allocation)
__global__ __launch_bounds__(256) void k_ilv(vec4* __restrict__ buf, uint32_t g) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t lo = j & ((1ull << g) - 1);
  const uint64_t c = ((j - lo) << 1) | lo;
  vec4 x = ld(buf + c), y = ld(buf + c + (1ull << g));
  st(buf + c, x * 1.0000001f);
  st(buf + c + (1ull << g), y * 0.9999999f);
}

// one-state pair kernel (the q1 apply row pattern at chunk bit lb)
__global__ __launch_bounds__(256) void k_pair1(vec4* __restrict__ f, uint32_t lb) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t lo = j & ((1ull << lb) - 1);
  const uint64_t c0 = ((j - lo) << 1) | lo, c1 = c0 + (1ull << lb);
  vec4 x0 = ld(f + c0), x1 = ld(f + c1);
  st(f + c0, x0 * 1.0000001f);
  st(f + c1, x1 * 1.0000001f);
}

// one-state quad: chunks c0 + {0, 2^lb, 2^lb2, 2^lb + 2^lb2}, lb2 < lb (a far pair split over a
// second, near "bank" bit)
__global__ __launch_bounds__(256) void k_quad1(vec4* __restrict__ f, uint32_t lb, uint32_t lb2) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t lo = j & ((1ull << lb2) - 1);
  uint64_t c0 = ((j - lo) << 1) | lo;
  lo = c0 & ((1ull << lb) - 1);
  c0 = ((c0 - lo) << 1) | lo;
  const uint64_t o[4] = {0, 1ull << lb2, 1ull << lb, (1ull << lb) + (1ull << lb2)};
  vec4 x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = ld(f + c0 + o[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) st(f + c0 + o[k], x[k] * 1.0000001f);
}

// one-state pair with the block order swizzled: block b runs item block b ^ (b >> s & m)
__global__ __launch_bounds__(256) void k_pair1s(vec4* __restrict__ f, uint32_t lb, uint32_t sh, uint32_t m) {
  const uint64_t bb = blockIdx.x ^ ((blockIdx.x >> sh) & m);
  const uint64_t j = bb * 256 + threadIdx.x;
  const uint64_t lo = j & ((1ull << lb) - 1);
  const uint64_t c0 = ((j - lo) << 1) | lo, c1 = c0 + (1ull << lb);
  vec4 x0 = ld(f + c0), x1 = ld(f + c1);
  st(f + c0, x0 * 1.0000001f);
  st(f + c1, x1 * 1.0000001f);
}

// two-state, block-contiguous: block b owns items [b*256*it, (b+1)*256*it), U in flight
template <int U>
__global__ __launch_bounds__(256) void k_blk2(vec4* __restrict__ f, vec4* __restrict__ b, uint32_t it) {
  const uint64_t start = (uint64_t)blockIdx.x * 256 * it + threadIdx.x;
  for (uint32_t s = 0; s < it; s += U) {
    vec4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = ld(f + start + (uint64_t)(s + u) * 256);
      y[u] = ld(b + start + (uint64_t)(s + u) * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st(f + start + (uint64_t)(s + u) * 256, x[u] * 1.0000001f);
      st(b + start + (uint64_t)(s + u) * 256, y[u] * 0.9999999f);
    }
  }
}
// two-state, grid-strided over 256-item blocks: round s of block b runs item block s*grid + b
// (the resident blocks sweep one contiguous window together)
template <int U>
__global__ __launch_bounds__(256) void k_win2(vec4* __restrict__ f, vec4* __restrict__ b, uint32_t it) {
  for (uint32_t s = 0; s < it; s += U) {
    vec4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = ((uint64_t)(s + u) * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
      x[u] = ld(f + i);
      y[u] = ld(b + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = ((uint64_t)(s + u) * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
      st(f + i, x[u] * 1.0000001f);
      st(b + i, y[u] * 0.9999999f);
    }
  }
}

// one state of an interleaved pair (every other 2^g-chunk block of the buffer)
__global__ __launch_bounds__(256) void k_ilv1(vec4* __restrict__ buf, uint32_t g) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t lo = j & ((1ull << g) - 1);
  const uint64_t c = ((j - lo) << 1) | lo;
  st(buf + c, ld(buf + c) * 1.0000001f);
}

template <int NS>
__global__ __launch_bounds__(256) void k_rmw(vec4* __restrict__ f, vec4* __restrict__ b) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  vec4 x = ld(f + i), y;
  if (NS == 2) y = ld(b + i);
  st(f + i, x * 1.0000001f);
  if (NS == 2) st(b + i, y * 0.9999999f);
}

static hipEvent_t e0, e1;
template <class F>
static float timeit(F fn, int reps = 5) {
  fn();
  CK(hipDeviceSynchronize());
  std::vector<float> v;
  for (int k = 0; k < 5; ++k) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    v.push_back(ms / reps);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const uint64_t nch = (1ull << 28) / 2;  // n = 28 f32: 2 GiB
  const size_t S = nch * 16;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t grid = (uint32_t)(nch / 256);
  auto tb2 = [&](vec4* f, vec4* b) {
    return 4.0 * S / timeit([&] { k_rmw<2><<<grid, 256>>>(f, b); }) / 1e9;
  };
  auto tb1 = [&](vec4* f) { return 2.0 * S / timeit([&] { k_rmw<1><<<grid, 256>>>(f, f); }) / 1e9; };
  for (int trial = 0; trial < 4; ++trial) {
    vec4 *fa, *ba;
    CK(hipMalloc(&fa, S));
    CK(hipMalloc(&ba, S));
    CK(hipMemset(fa, 0, S));
    CK(hipMemset(ba, 0, S));
    printf("trial %d 2-state blk (it:TB/s):", trial);
    for (uint32_t it : {1u, 2u, 4u, 8u, 16u, 64u, 256u})
      printf(" %u:%.2f", it, 4.0 * S / timeit([&] { k_blk2<1><<<grid / it, 256>>>(fa, ba, it); }) / 1e9);
    printf("  U2:");
    for (uint32_t it : {2u, 8u, 64u, 256u})
      printf(" %u:%.2f", it, 4.0 * S / timeit([&] { k_blk2<2><<<grid / it, 256>>>(fa, ba, it); }) / 1e9);
    printf("  win (it):");
    for (uint32_t it : {4u, 16u, 64u, 256u})
      printf(" %u:%.2f", it, 4.0 * S / timeit([&] { k_win2<1><<<grid / it, 256>>>(fa, ba, it); }) / 1e9);
    printf("  ilv1 (g):");
    {
      vec4* buf;
      CK(hipMalloc(&buf, 2 * S));
      CK(hipMemset(buf, 0, 2 * S));
      for (uint32_t g : {10u, 12u, 14u})
        printf(" %u:%.2f/%.2f", g, 2.0 * S / timeit([&] { k_ilv1<<<grid, 256>>>(buf, g); }) / 1e9,
               4.0 * S / timeit([&] { k_ilv<<<grid, 256>>>(buf, g); }) / 1e9);
      CK(hipFree(buf));
    }
    printf("  winU2:");
    for (uint32_t it : {64u, 256u})
      printf(" %u:%.2f", it, 4.0 * S / timeit([&] { k_win2<2><<<grid / it, 256>>>(fa, ba, it); }) / 1e9);
    printf("\n");
    fflush(stdout);
    CK(hipFree(fa));
    CK(hipFree(ba));
  }
  return 0;
}
