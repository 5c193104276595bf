// Two-state in-place streaming probe (timing tool, not product).  The single-gate reverse
// kernels read and write two 2 GiB states (fwd, bwd) at the same indices and measure 63-65 %
// of 8 TB/s, the one-state kernels 75-82 %.  This isolates the memory pattern from the gate
// math: every kernel here is the diagonal-gate skeleton (k_diag in csrc/qdc_kernels.hpp) with a
// scale in place of the gate.
//   variants: cache policy of loads / stores (nt or default), items in flight per thread (U),
//   block-contiguous vs grid-strided iteration, relative placement of the two states (separate
//   allocations, one allocation with pads), and a "phase" split where fwd and bwd accesses of
//   one block are half a block range apart in time.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/twostate tools/twostate_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <int NT>
__device__ __forceinline__ vec4 ld(const vec4* p) {
  if constexpr (NT) return __builtin_nontemporal_load((const gvec4*)p);
  else return *(const gvec4*)p;
}
template <int NT>
__device__ __forceinline__ void st(vec4* p, vec4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, (gvec4*)p);
  else *(gvec4*)p = v;
}

// NS states, U chunks per thread in flight; block b owns [b*256*it, (b+1)*256*it) (ORDER 0) or
// grid-strided items (ORDER 1).  LNT/SNT: nontemporal loads/stores.
template <int NS, int U, int LNT, int SNT, int ORDER>
__global__ __launch_bounds__(256) void k_rmw(vec4* __restrict__ f, vec4* __restrict__ b,
                                              uint64_t n, uint32_t it) {
  if constexpr (ORDER == 0) {
    const uint64_t start = (uint64_t)blockIdx.x * 256 * it + threadIdx.x;
    for (uint32_t s = 0; s < it; s += U) {
      vec4 x[U], y[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = start + (uint64_t)(s + u) * 256;
        x[u] = ld<LNT>(f + i);
        if (NS == 2) y[u] = ld<LNT>(b + i);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = start + (uint64_t)(s + u) * 256;
        st<SNT>(f + i, x[u] * 1.0000001f);
        if (NS == 2) st<SNT>(b + i, y[u] * 0.9999999f);
      }
    }
  } else {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
      vec4 x[U], y[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = ld<LNT>(f + i0 + (uint64_t)u * 256);
        if (NS == 2) y[u] = ld<LNT>(b + i0 + (uint64_t)u * 256);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        st<SNT>(f + i0 + (uint64_t)u * 256, x[u] * 1.0000001f);
        if (NS == 2) st<SNT>(b + i0 + (uint64_t)u * 256, y[u] * 0.9999999f);
      }
    }
  }
}

// fwd chunks of a step first (loads + stores), then bwd chunks: per wave the two streams are
// not interleaved instruction by instruction.
template <int U>
__global__ __launch_bounds__(256) void k_rmw_seq(vec4* __restrict__ f, vec4* __restrict__ b,
                                                  uint64_t n, uint32_t it) {
  const uint64_t start = (uint64_t)blockIdx.x * 256 * it + threadIdx.x;
  for (uint32_t s = 0; s < it; s += U) {
    vec4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = ld<1>(f + start + (uint64_t)(s + u) * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) y[u] = ld<1>(b + start + (uint64_t)(s + u) * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st<1>(f + start + (uint64_t)(s + u) * 256, x[u] * 1.0000001f);
#pragma unroll
    for (int u = 0; u < U; ++u) st<1>(b + start + (uint64_t)(s + u) * 256, y[u] * 0.9999999f);
  }
}

// Two-state in-place with the two states' stores deferred by one step (stores of step s-1
// issued after the loads of step s): the write stream trails the read stream.
template <int U>
__global__ __launch_bounds__(256) void k_rmw_pipe(vec4* __restrict__ f, vec4* __restrict__ b,
                                                   uint64_t n, uint32_t it) {
  const uint64_t start = (uint64_t)blockIdx.x * 256 * it + threadIdx.x;
  vec4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = ld<1>(f + start + (uint64_t)u * 256);
    y[u] = ld<1>(b + start + (uint64_t)u * 256);
  }
  for (uint32_t s = 0; s < it; s += U) {
    vec4 xn[U], yn[U];
    const bool more = s + U < it;
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xn[u] = ld<1>(f + start + (uint64_t)(s + U + u) * 256);
        yn[u] = ld<1>(b + start + (uint64_t)(s + U + u) * 256);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st<1>(f + start + (uint64_t)(s + u) * 256, x[u] * 1.0000001f);
      st<1>(b + start + (uint64_t)(s + u) * 256, y[u] * 0.9999999f);
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x[u] = xn[u];
        y[u] = yn[u];
      }
    }
  }
}

__global__ void k_copy(const vec4* __restrict__ s, vec4* __restrict__ d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    st<1>(d + i, ld<1>(s + i));
}

static hipEvent_t e0, e1;
template <class F>
static float timeit(F fn, int reps = 5) {
  fn();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int k = 0; k < 3; ++k) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms / reps);
  }
  return best;
}

int main(int argc, char** argv) {
  const uint64_t nch = (1ull << 28) / 2;  // 16-B chunks of an n = 28 f32 state (2 GiB)
  const double S = (double)nch * 16;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  vec4 *f, *b, *c;
  CK(hipMalloc(&f, nch * 16));
  CK(hipMalloc(&b, nch * 16));
  CK(hipMalloc(&c, nch * 16));
  CK(hipMemset(f, 0, nch * 16));
  CK(hipMemset(b, 0, nch * 16));
  CK(hipMemset(c, 0, nch * 16));
  printf("f=%p b=%p c=%p\n", (void*)f, (void*)b, (void*)c);
  auto rep = [&](const char* name, double bytes, float ms) {
    printf("%-48s %7.3f ms %6.2f TB/s %5.1f%%\n", name, ms, bytes / ms / 1e9, bytes / ms / 1e9 / 80.0);
  };
  rep("copy nt", 2 * S, timeit([&] { k_copy<<<cus * 32, 256>>>(f, c, nch); }));
  // block-contiguous like k_direct / k_diag: it items per thread, grid = nch / (256 * it)
  for (uint32_t it : {16u, 64u, 256u}) {
    const uint32_t grid = (uint32_t)(nch / (256ull * it));
    char nm[96];
    snprintf(nm, sizeof nm, "1st rmw nt/nt U=4 blk it=%u", it);
    rep(nm, 2 * S, timeit([&] { k_rmw<1, 4, 1, 1, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw nt/nt U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 1, 1, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw nt/nt U=8 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 8, 1, 1, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw nt/nt U=2 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 2, 1, 1, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw def/nt U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 0, 1, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw nt/def U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 1, 0, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st rmw def/def U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 0, 0, 0><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st seq U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw_seq<4><<<grid, 256>>>(f, b, nch, it); }));
    snprintf(nm, sizeof nm, "2st pipe U=4 blk it=%u", it);
    rep(nm, 4 * S, timeit([&] { k_rmw_pipe<4><<<grid, 256>>>(f, b, nch, it); }));
  }
  for (int gm : {4, 8, 16}) {
    char nm[96];
    snprintf(nm, sizeof nm, "2st rmw nt/nt U=4 grid-stride %d/CU", gm);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 1, 1, 1><<<cus * gm, 256>>>(f, b, nch, 0); }));
  }
  // one allocation, b = f + S + pad
  vec4* base;
  const size_t maxpad = (size_t)64 << 20;
  CK(hipMalloc(&base, 2 * nch * 16 + maxpad));
  CK(hipMemset(base, 0, 2 * nch * 16 + maxpad));
  const size_t pads[] = {0, 256, 2048, 4096, 8192, 65536, (size_t)1 << 20, ((size_t)1 << 21) + 4096,
                         ((size_t)32 << 20) + 8192};
  const uint32_t it = 64, grid = (uint32_t)(nch / (256ull * it));
  for (size_t pad : pads) {
    vec4* ff = base;
    vec4* bb = base + (nch * 16 + pad) / 16;
    char nm[96];
    snprintf(nm, sizeof nm, "2st rmw U=4 it=64 one alloc pad %zu", pad);
    rep(nm, 4 * S, timeit([&] { k_rmw<2, 4, 1, 1, 0><<<grid, 256>>>(ff, bb, nch, it); }));
  }
  // fwd and bwd at the SAME buffer halves swapped (b before f)
  {
    vec4* ff = base + (nch * 16 + 4096) / 16;
    vec4* bb = base;
    rep("2st rmw U=4 it=64 b below f (pad 4096)", 4 * S,
        timeit([&] { k_rmw<2, 4, 1, 1, 0><<<grid, 256>>>(ff, bb, nch, it); }));
  }
  return 0;
}
