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
    vec4 *ini, *st_, *bwd;
    CK(hipMalloc(&ini, S));
    CK(hipMalloc(&st_, S));
    CK(hipMemset(ini, 0, S));
    CK(hipMemset(st_, 0, S));
    CK(hipMalloc(&bwd, S));
    CK(hipMemset(bwd, 0, S));
    const long long d1 = (long long)((char*)bwd - (char*)st_);
    printf("trial %d pair strides (chunk bit: TB/s):", trial);
    for (uint32_t lb : {6u, 9u, 10u, 11u, 12u, 13u, 14u, 16u, 20u})
      printf(" %u:%.2f", lb,
             4.0 * S / timeit([&] { k_pair<<<grid / 2, 256>>>(st_, bwd, lb); }) / 1e9);
    printf("\n");
    printf("trial %d quad lb=6, lb2:", trial);
    for (uint32_t lb2 : {9u, 10u, 11u, 12u, 13u, 14u, 16u})
      printf(" %u:%.2f", lb2,
             4.0 * S / timeit([&] { k_quad<<<grid / 4, 256>>>(st_, bwd, 6, lb2); }) / 1e9);
    printf("\n");
    printf("trial %d quad lb=16, lb2:", trial);
    for (uint32_t lb2 : {17u, 18u, 20u, 24u})
      printf(" %u:%.2f", lb2,
             4.0 * S / timeit([&] { k_quad<<<grid / 4, 256>>>(st_, bwd, 16, lb2); }) / 1e9);
    printf("\n");
    printf("trial %d ini %p st %p bwd %p (bwd-st %+lld MiB)  1st: st %.2f bwd %.2f  "
           "2st: st/bwd %.2f ini/st %.2f ini/bwd %.2f TB/s\n",
           trial, (void*)ini, (void*)st_, (void*)bwd, d1 >> 20, tb1(st_), tb1(bwd), tb2(st_, bwd),
           tb2(ini, st_), tb2(ini, bwd));
    fflush(stdout);
    CK(hipFree(bwd));
    CK(hipFree(st_));
    CK(hipFree(ini));
  }
  for (int trial = 0; trial < 4; ++trial) {
    vec4* buf;
    CK(hipMalloc(&buf, 2 * S));
    CK(hipMemset(buf, 0, 2 * S));
    printf("trial %d interleaved 2-state (g: TB/s):", trial);
    for (uint32_t g : {6u, 8u, 10u, 12u, 14u, 16u, 17u, 20u})
      printf(" %u:%.2f", g, 4.0 * S / timeit([&] { k_ilv<<<grid, 256>>>(buf, g); }) / 1e9);
    printf("  split halves: %.2f\n", tb2(buf, buf + nch));
    printf("trial %d one-state pairs in the first half (chunk bit: TB/s):", trial);
    for (uint32_t lb = 0; lb < 27; ++lb)
      printf(" %u:%.2f", lb, 2.0 * S / timeit([&] { k_pair1<<<grid / 2, 256>>>(buf, lb); }) / 1e9);
    printf("\n");
    fflush(stdout);
    CK(hipFree(buf));
  }
  return 0;
}
