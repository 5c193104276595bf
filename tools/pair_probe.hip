// Pair-stream probe (timing tool, not product).  Two questions behind the single-gate rows of
// bench.py --micro:
//  1. the two-state reverse shape (rows c0, c0 + 2^lb of fwd and bwd, in place) on two separate
//     allocations vs one buffer holding fwd and bwd interleaved in 2^g-chunk blocks, over
//     several allocation trials (placement churn between trials);
//  2. the one-state far-pair shape (apply_q1 at chunk bits 20..25) with 1, 2 or 4 items in
//     flight per thread, block-contiguous or grid-strided.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/pair_probe tools/pair_probe.hip
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
__device__ __forceinline__ uint64_t ins0(uint64_t x, uint32_t b) {
  const uint64_t lo = x & ((1ull << b) - 1);
  return ((x - lo) << 1) | lo;
}

// two-state pair; state chunk c lives at c + (c & gm) (gm = ~(2^g - 1): interleaved, 0: not);
// bwd = f + boff
__global__ __launch_bounds__(256) void k_pair2(vec4* __restrict__ f, uint64_t boff, uint32_t lb,
                                               uint64_t gm) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t c0 = ins0(j, lb), c1 = c0 + (1ull << lb);
  c0 += c0 & gm;
  c1 += c1 & gm;
  vec4* b = f + boff;
  vec4 x0 = ld(f + c0), x1 = ld(f + c1), y0 = ld(b + c0), y1 = ld(b + c1);
  st(f + c0, x0 * 1.0000001f);
  st(f + c1, x1 * 1.0000001f);
  st(b + c0, y0 * 0.9999999f);
  st(b + c1, y1 * 0.9999999f);
}

// one-state far pair, U items per thread: block-contiguous (MODE 0: block b owns items
// [b*256*U, ...)) or grid-strided (MODE 1: item u*grid*256 + b*256 + t)
template <int U, int MODE>
__global__ __launch_bounds__(256) void k_far(vec4* __restrict__ f, uint32_t lb) {
  vec4 x0[U], x1[U];
  uint64_t c0[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t j = MODE == 0 ? ((uint64_t)blockIdx.x * U + u) * 256 + threadIdx.x
                                 : ((uint64_t)u * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
    c0[u] = ins0(j, lb);
    x0[u] = ld(f + c0[u]);
    x1[u] = ld(f + c0[u] + (1ull << lb));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    st(f + c0[u], x0[u] * 1.0000001f);
    st(f + c0[u] + (1ull << lb), x1[u] * 1.0000001f);
  }
}

static hipEvent_t e0, e1;
template <class F>
static float timeit(F fn, int reps = 4) {
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
  const uint64_t nch = (1ull << 28) / 2;  // n = 28 f32: 2 GiB per state
  const size_t S = nch * 16;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t grid = (uint32_t)(nch / 2 / 256);
  const uint32_t lbs[] = {0, 1, 4, 9, 13, 18, 22, 25};
  for (int trial = 0; trial < 6; ++trial) {
    // placement churn: a pad of trial-dependent size stays allocated during the trial
    void* pad = nullptr;
    CK(hipMalloc(&pad, ((size_t)(trial * 7 % 5) + 1) << 28));
    vec4 *fa, *ba, *buf;
    CK(hipMalloc(&fa, S));
    CK(hipMalloc(&ba, S));
    CK(hipMalloc(&buf, 2 * S));
    CK(hipMemset(fa, 0, S));
    CK(hipMemset(ba, 0, S));
    CK(hipMemset(buf, 0, 2 * S));
    printf("trial %d separate (lb:TB/s):", trial);
    for (uint32_t lb : lbs)
      printf(" %u:%.2f", lb,
             4.0 * S / timeit([&] { k_pair2<<<grid, 256>>>(fa, (uint64_t)(ba - fa), lb, 0); }) / 1e9);
    printf("\n  one alloc bwd=f+S:");
    for (uint32_t lb : lbs)
      printf(" %u:%.2f", lb,
             4.0 * S / timeit([&] { k_pair2<<<grid, 256>>>(buf, nch, lb, 0); }) / 1e9);
    for (uint32_t g : {10u, 12u}) {
      printf("\n  interleaved g=%u:", g);
      const uint64_t gm = ~((1ull << g) - 1);
      for (uint32_t lb : lbs)
        printf(" %u:%.2f", lb,
               4.0 * S / timeit([&] { k_pair2<<<grid, 256>>>(buf, 1ull << g, lb, gm); }) / 1e9);
    }
    printf("\n  one-state far (lb: U1b U2b U4b U2g U4g):");
    for (uint32_t lb : {12u, 20u, 21u, 22u, 23u, 24u, 25u}) {
      printf(" %u:", lb);
      printf("%.2f/", 2.0 * S / timeit([&] { k_far<1, 0><<<grid, 256>>>(fa, lb); }) / 1e9);
      printf("%.2f/", 2.0 * S / timeit([&] { k_far<2, 0><<<grid / 2, 256>>>(fa, lb); }) / 1e9);
      printf("%.2f/", 2.0 * S / timeit([&] { k_far<4, 0><<<grid / 4, 256>>>(fa, lb); }) / 1e9);
      printf("%.2f/", 2.0 * S / timeit([&] { k_far<2, 1><<<grid / 2, 256>>>(fa, lb); }) / 1e9);
      printf("%.2f", 2.0 * S / timeit([&] { k_far<4, 1><<<grid / 4, 256>>>(fa, lb); }) / 1e9);
    }
    printf("\n");
    fflush(stdout);
    CK(hipFree(fa));
    CK(hipFree(ba));
    CK(hipFree(buf));
    CK(hipFree(pad));
  }
  return 0;
}
