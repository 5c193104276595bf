// bw_probe.hip — HBM streaming configuration probe for the state-vector kernels (gfx950).
// Variants: grid size (persistent grid-stride vs one-shot), items in flight per thread,
// nontemporal loads/stores, and a 1-qubit pair kernel at several target strides.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
struct alignas(16) c4 {
  float x, y, z, w;
};

template <typename T>
__device__ __forceinline__ T ld(const T* p, bool nt) {
  if (nt) return __builtin_nontemporal_load(p);
  return *p;
}
template <typename T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// copy with U chunks per thread per iteration, grid-stride
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4f* __restrict__ a, v4f* __restrict__ b,
                                              uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n) v[u] = NT ? __builtin_nontemporal_load(a + base + u * 256) : a[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * 256 < n) {
        if (NT)
          __builtin_nontemporal_store(v[u], b + base + u * 256);
        else
          b[base + u * 256] = v[u];
      }
  }
}

__device__ __forceinline__ uint64_t insert_zero(uint64_t x, uint32_t b) {
  const uint64_t low = x & ((1ull << b) - 1ull);
  return ((x - low) << 1) | low;
}

// in-place 1q gate on v4f chunks (2 complex each), pair stride 2^p chunks, U pairs per thread
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_q1(v4f* __restrict__ s, float g0, float g1, float g2,
                                            float g3, uint32_t p, uint64_t items) {
  const uint64_t off = 1ull << p;
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; base < items;
       base += stride) {
    v4f a[U], b[U];
    uint64_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = insert_zero(base + u * 256, p);
      a[u] = NT ? __builtin_nontemporal_load(s + c[u]) : s[c[u]];
      b[u] = NT ? __builtin_nontemporal_load(s + c[u] + off) : s[c[u] + off];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v4f x = a[u], y = b[u];
      v4f o0 = {g0 * x.x + g1 * y.x, g0 * x.y + g1 * y.y, g0 * x.z + g1 * y.z, g0 * x.w + g1 * y.w};
      v4f o1 = {g2 * x.x + g3 * y.x, g2 * x.y + g3 * y.y, g2 * x.z + g3 * y.z, g2 * x.w + g3 * y.w};
      if (NT) {
        __builtin_nontemporal_store(o0, s + c[u]);
        __builtin_nontemporal_store(o1, s + c[u] + off);
      } else {
        s[c[u]] = o0;
        s[c[u] + off] = o1;
      }
    }
  }
}


// one-shot (no grid-stride loop) variants: each thread handles U items exactly once
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_q1_once(v4f* __restrict__ s, float g0, float g1, float g2,
                                                 float g3, uint32_t p, uint64_t items) {
  const uint64_t off = 1ull << p;
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f a[U], b[U];
  uint64_t c[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    c[u] = insert_zero(base + u * 256, p);
    if (base + u * 256 < items) {
      a[u] = NT ? __builtin_nontemporal_load(s + c[u]) : s[c[u]];
      b[u] = NT ? __builtin_nontemporal_load(s + c[u] + off) : s[c[u] + off];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (base + u * 256 >= items) continue;
    v4f x = a[u], y = b[u];
    v4f o0 = g0 * x + g1 * y;
    v4f o1 = g2 * x + g3 * y;
    if (NT) {
      __builtin_nontemporal_store(o0, s + c[u]);
      __builtin_nontemporal_store(o1, s + c[u] + off);
    } else {
      s[c[u]] = o0;
      s[c[u] + off] = o1;
    }
  }
}

// fused two-state pass (like the reverse sweep): f and b pairs, in place
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_rev_once(v4f* __restrict__ f, v4f* __restrict__ bb,
                                                  float g0, float g1, uint32_t p, uint64_t items) {
  const uint64_t off = 1ull << p;
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f a[U], b[U], x[U], y[U];
  uint64_t c[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    c[u] = insert_zero(base + u * 256, p);
    if (base + u * 256 < items) {
      a[u] = NT ? __builtin_nontemporal_load(f + c[u]) : f[c[u]];
      b[u] = NT ? __builtin_nontemporal_load(f + c[u] + off) : f[c[u] + off];
      x[u] = NT ? __builtin_nontemporal_load(bb + c[u]) : bb[c[u]];
      y[u] = NT ? __builtin_nontemporal_load(bb + c[u] + off) : bb[c[u] + off];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (base + u * 256 >= items) continue;
    v4f o0 = g0 * a[u] + g1 * b[u], o1 = g1 * a[u] - g0 * b[u];
    v4f p0 = g0 * x[u] - g1 * y[u], p1 = g1 * x[u] + g0 * y[u];
    if (NT) {
      __builtin_nontemporal_store(o0, f + c[u]);
      __builtin_nontemporal_store(o1, f + c[u] + off);
      __builtin_nontemporal_store(p0, bb + c[u]);
      __builtin_nontemporal_store(p1, bb + c[u] + off);
    } else {
      f[c[u]] = o0; f[c[u] + off] = o1; bb[c[u]] = p0; bb[c[u] + off] = p1;
    }
  }
}


// block-contiguous: block b owns items [b*256*IT, (b+1)*256*IT), U items in flight per step
template <int IT, int U, bool NT>
__global__ __launch_bounds__(256) void k_rev_blk(v4f* __restrict__ f, v4f* __restrict__ bb,
                                                 float g0, float g1, uint32_t p, uint64_t items,
                                                 float* __restrict__ part) {
  const uint64_t off = 1ull << p;
  const uint64_t b0 = (uint64_t)blockIdx.x * 256 * IT + threadIdx.x;
  v4f acc = {0, 0, 0, 0};
  for (int it = 0; it < IT; it += U) {
    v4f a[U], b[U], x[U], y[U];
    uint64_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = insert_zero(b0 + (uint64_t)(it + u) * 256, p);
      a[u] = NT ? __builtin_nontemporal_load(f + c[u]) : f[c[u]];
      b[u] = NT ? __builtin_nontemporal_load(f + c[u] + off) : f[c[u] + off];
      x[u] = NT ? __builtin_nontemporal_load(bb + c[u]) : bb[c[u]];
      y[u] = NT ? __builtin_nontemporal_load(bb + c[u] + off) : bb[c[u] + off];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v4f o0 = g0 * a[u] + g1 * b[u], o1 = g1 * a[u] - g0 * b[u];
      acc += x[u] * o0 + y[u] * o1;
      v4f p0 = g0 * x[u] - g1 * y[u], p1 = g1 * x[u] + g0 * y[u];
      if (NT) {
        __builtin_nontemporal_store(o0, f + c[u]);
        __builtin_nontemporal_store(o1, f + c[u] + off);
        __builtin_nontemporal_store(p0, bb + c[u]);
        __builtin_nontemporal_store(p1, bb + c[u] + off);
      } else {
        f[c[u]] = o0; f[c[u] + off] = o1; bb[c[u]] = p0; bb[c[u] + off] = p1;
      }
    }
  }
  // cheap block partial (one value) to keep acc live
  float v = acc.x + acc.y + acc.z + acc.w;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = v;
}

// read-only density-like reduction, block-contiguous
template <int IT, int U, bool NT>
__global__ __launch_bounds__(256) void k_red_blk(const v4f* __restrict__ s, uint32_t p, uint64_t items,
                                                 float* __restrict__ part) {
  const uint64_t off = 1ull << p;
  const uint64_t b0 = (uint64_t)blockIdx.x * 256 * IT + threadIdx.x;
  v4f acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  for (int it = 0; it < IT; it += U) {
    v4f a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t c = insert_zero(b0 + (uint64_t)(it + u) * 256, p);
      a[u] = NT ? __builtin_nontemporal_load(s + c) : s[c];
      b[u] = NT ? __builtin_nontemporal_load(s + c + off) : s[c + off];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { acc0 += a[u] * a[u]; acc1 += a[u] * b[u]; }
  }
  float v = acc0.x + acc0.y + acc0.z + acc0.w + acc1.x + acc1.y + acc1.z + acc1.w;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = v;
}


// reverse with f/b interleaved in blocks of 2^gb chunks: f block k at 2k, b block k at 2k+1
template <int U>
__global__ __launch_bounds__(256) void k_rev_il(v4f* __restrict__ base, float g0, float g1, uint32_t p,
                                                uint32_t gb, uint64_t items) {
  const uint64_t off = 1ull << p;
  const uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  const uint64_t gm = (1ull << gb) - 1;
  auto fa = [&](uint64_t c) { return ((c >> gb) << (gb + 1)) | (c & gm); };
  v4f a[U], b[U], x[U], y[U];
  uint64_t c[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    c[u] = insert_zero(i0 + u * 256, p);
    a[u] = __builtin_nontemporal_load(base + fa(c[u]));
    b[u] = __builtin_nontemporal_load(base + fa(c[u] + off));
    x[u] = __builtin_nontemporal_load(base + fa(c[u]) + (1ull << gb));
    y[u] = __builtin_nontemporal_load(base + fa(c[u] + off) + (1ull << gb));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    v4f o0 = g0 * a[u] + g1 * b[u], o1 = g1 * a[u] - g0 * b[u];
    v4f p0 = g0 * x[u] - g1 * y[u], p1 = g1 * x[u] + g0 * y[u];
    __builtin_nontemporal_store(o0, base + fa(c[u]));
    __builtin_nontemporal_store(o1, base + fa(c[u] + off));
    __builtin_nontemporal_store(p0, base + fa(c[u]) + (1ull << gb));
    __builtin_nontemporal_store(p1, base + fa(c[u] + off) + (1ull << gb));
  }
}

template <typename K, typename... A>
float timeit(K k, int grid, int reps, A... args) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, args...);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, args...);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int nq = argc > 1 ? atoi(argv[1]) : 28;
  const uint64_t amps = 1ull << nq;
  const uint64_t nch = amps / 2;  // v4f chunks
  const uint64_t items = nch / 2;
  const double bytes = (double)amps * 8;
  const int reps = 10;
  float* part;
  CK(hipMalloc(&part, sizeof(float) * 4 * (items / 256 + 1)));
  printf("state %.2f GiB\n", bytes / (1 << 30));
  auto rev = [&](v4f* x, v4f* y) {
    int g = (int)(items / (256 * 2));
    return 4 * bytes / timeit(k_rev_once<2, true>, g, reps, x, y, 0.6f, 0.8f, 8u, items) / 1e6;
  };
  auto cpy = [&](v4f* x, v4f* y) {
    int g = (int)(nch / 256);
    return 2 * bytes / timeit(k_copy<1, true>, g, reps, (const v4f*)x, y, nch) / 1e6;
  };
  auto q1 = [&](v4f* x) {
    int g = (int)(items / 256);
    return 2 * bytes / timeit(k_q1_once<1, true>, g, reps, x, 0.6f, 0.8f, -0.8f, 0.6f, 8u, items) / 1e6;
  };
  std::vector<v4f*> keep;
  for (int rep = 0; rep < 6; ++rep) {
    v4f *x, *y;
    CK(hipMalloc(&x, bytes));
    CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0, bytes));
    CK(hipMemset(y, 0, bytes));
    keep.push_back(x);
    keep.push_back(y);
    printf("pair %d x=%p y=%p : rev %.0f %.0f %.0f | copy xy %.0f yx %.0f | q1 x %.0f y %.0f GB/s\n", rep,
           (void*)x, (void*)y, rev(x, y), rev(x, y), rev(y, x), cpy(x, y), cpy(y, x), q1(x), q1(y));
  }
  // cross pairs: buffer i with buffer j
  printf("cross rev: ");
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      if (i != j) printf("(%d,%d) %.0f ", i, j, rev(keep[i], keep[j]));
  printf("\n");
  for (auto p : keep) CK(hipFree(p));
  printf("--- interleaved f/b layout ---\n");
  {
    v4f* big;
    CK(hipMalloc(&big, 2 * bytes));
    CK(hipMemset(big, 0, 2 * bytes));
    for (uint32_t gb : {6u, 8u, 10u, 12u, 14u, 16u, 20u}) {
      int g = (int)(items / (256 * 2));
      float ms = timeit(k_rev_il<2>, g, reps, big, 0.6f, 0.8f, 8u, gb, items);
      float ms2 = timeit(k_rev_il<2>, g, reps, big, 0.6f, 0.8f, 20u, gb, items);
      printf("interleave gb %2u (%8u B) : p8 %.1f p20 %.1f GB/s | halves rev %.0f\n", gb, (16u << gb),
             4 * bytes / ms / 1e6, 4 * bytes / ms2 / 1e6, rev(big, (v4f*)((char*)big + (size_t)bytes)));
    }
  }
  return 0;
}
