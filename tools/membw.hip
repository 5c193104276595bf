// Memory-pattern probe for the fused passes' load/store skeleton (timing tool, not product).
// In-place read-modify-write of one or two 2 GiB states (n = 28 f32) in tile patterns:
//   tile = 2^T 16-B chunks: `lc` contiguous low chunk bits, the rest "row" bits at chunk
//   positions rb[0..]; thread bits = tile bits 0..log2(NT)-1, each thread 8 chunks (the top 3
//   tile bits), like k_rq's HBM layout.  persistent: a resident grid walks tiles (block-
//   contiguous or grid-strided); else one tile per block.
// Also plain streaming kernels (copy, in-place RMW) as the reference rates.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/membw tools/membw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
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
__device__ __forceinline__ uint64_t insert_zero(uint64_t x, uint32_t b) {
  const uint64_t lo = x & ((1ull << b) - 1);
  return ((x >> b) << (b + 1)) | lo;
}

struct geo {
  unsigned long long* ctr;  // work queue: [0] next tile, [1] finished blocks
  uint64_t ntiles;
  uint32_t lc, h, hb[8];
  uint32_t tpb;    // tiles per block (persistent)
  uint32_t order;  // 0 block-contiguous, 1 grid-strided
};

// NS states, NT threads, 8 chunks per thread and state; tile = NT * 8 chunks
template <int NS, int NT>
__global__ __launch_bounds__(NT) void k_tile(vec4* __restrict__ f, vec4* __restrict__ b, geo g,
                                              uint32_t persistent) {
  constexpr int LOGNT = NT == 128 ? 7 : 8;
  const uint32_t t = threadIdx.x;
  // chunk offset of thread bit k / register bit i within the tile (tile bit -> global chunk bit)
  auto gbit = [&](uint32_t tb) -> uint64_t {
    return tb < g.lc ? (1ull << tb) : (1ull << g.hb[tb - g.lc]);
  };
  uint64_t thr = 0;
  for (int k = 0; k < LOGNT; ++k)
    if ((t >> k) & 1u) thr += gbit((uint32_t)k);
  uint64_t offi[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t o = 0;
    for (int s = 0; s < 3; ++s)
      if ((i >> s) & 1) o += gbit((uint32_t)(LOGNT + s));
    offi[i] = o;
  }
  auto base_of = [&](uint64_t tile) {
    uint64_t base = tile << g.lc;
    for (uint32_t k = 0; k < g.h; ++k) base = insert_zero(base, g.hb[k]);
    return base;
  };
  uint64_t t0, step, count;
  if (persistent == 2) {  // work queue: tiles handed out in order by an atomic counter
    __shared__ unsigned long long next;
    for (;;) {
      if (t == 0) next = atomicAdd(&g.ctr[0], 1ull);
      __syncthreads();
      const uint64_t tile = next;
      __syncthreads();
      if (tile >= g.ntiles) break;
      const uint64_t base = base_of(tile) + thr;
      vec4 x[NS][8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        x[0][i] = ld(f + base + offi[i]);
        if (NS == 2) x[NS - 1][i] = ld(b + base + offi[i]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        st(f + base + offi[i], x[0][i] * 1.0000001f);
        if (NS == 2) st(b + base + offi[i], x[NS - 1][i] * 0.9999999f);
      }
    }
    if (t == 0) {  // the last block to finish resets the queue for the next launch
      __threadfence();
      if (atomicAdd(&g.ctr[1], 1ull) == gridDim.x - 1) {
        g.ctr[0] = 0;
        g.ctr[1] = 0;
        __threadfence();
      }
    }
    return;
  }
  if (persistent) {
    t0 = g.order ? blockIdx.x : (uint64_t)blockIdx.x * g.tpb;
    step = g.order ? gridDim.x : 1;
    count = t0 >= g.ntiles ? 0 : g.order ? (g.ntiles - 1 - t0) / step + 1 : min((uint64_t)g.tpb, g.ntiles - t0);
  } else {
    t0 = blockIdx.x;
    step = 1;
    count = 1;
  }
  for (uint64_t s = 0; s < count; ++s) {
    const uint64_t base = base_of(t0 + s * step) + thr;
    vec4 x[NS][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      x[0][i] = ld(f + base + offi[i]);
      if (NS == 2) x[NS - 1][i] = ld(b + base + offi[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      x[0][i] *= 1.0000001f;
      st(f + base + offi[i], x[0][i]);
      if (NS == 2) {
        x[NS - 1][i] *= 0.9999999f;
        st(b + base + offi[i], x[NS - 1][i]);
      }
    }
  }
}

// streaming reference: U chunks per thread in flight, grid-stride over the state
template <int NS, int U>
__global__ __launch_bounds__(256) void k_stream(vec4* __restrict__ f, vec4* __restrict__ b,
                                                 uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    vec4 x[NS][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[0][u] = ld(f + i0 + (uint64_t)u * 256);
      if (NS == 2) x[NS - 1][u] = ld(b + i0 + (uint64_t)u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st(f + i0 + (uint64_t)u * 256, x[0][u] * 1.0000001f);
      if (NS == 2) st(b + i0 + (uint64_t)u * 256, x[NS - 1][u] * 0.9999999f);
    }
  }
}

__global__ void k_copy(const vec4* __restrict__ s, vec4* __restrict__ d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    st(d + i, ld(s + i));
}

static float timeit(hipEvent_t e0, hipEvent_t e1, void (*fn)(void*), void* arg, int reps) {
  fn(arg);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) fn(arg);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

struct Run {
  vec4 *f, *b;
  uint64_t n;
  geo g;
  int ns, nt, persistent, grid, mode, u;
};

static void launch(void* a) {
  Run& r = *(Run*)a;
  if (r.mode == 0) {
    k_copy<<<r.grid, 256>>>(r.f, r.b, r.n);
  } else if (r.mode == 1) {
    if (r.ns == 1 && r.u == 4) k_stream<1, 4><<<r.grid, 256>>>(r.f, r.b, r.n);
    if (r.ns == 1 && r.u == 8) k_stream<1, 8><<<r.grid, 256>>>(r.f, r.b, r.n);
    if (r.ns == 2 && r.u == 4) k_stream<2, 4><<<r.grid, 256>>>(r.f, r.b, r.n);
    if (r.ns == 2 && r.u == 8) k_stream<2, 8><<<r.grid, 256>>>(r.f, r.b, r.n);
  } else {
    const uint32_t grid = r.persistent ? (uint32_t)r.grid : (uint32_t)r.g.ntiles;
    if (r.ns == 1 && r.nt == 256) k_tile<1, 256><<<grid, 256>>>(r.f, r.b, r.g, r.persistent);
    if (r.ns == 1 && r.nt == 128) k_tile<1, 128><<<grid, 128>>>(r.f, r.b, r.g, r.persistent);
    if (r.ns == 2 && r.nt == 128) k_tile<2, 128><<<grid, 128>>>(r.f, r.b, r.g, r.persistent);
  }
}

int main(int argc, char** argv) {
  const int n = 28;
  const uint64_t nch = (1ull << n) / 2;  // 16-B chunks of an f32 state
  vec4 *f, *b, *c;
  CK(hipMalloc(&f, nch * 16));
  CK(hipMalloc(&b, nch * 16));
  CK(hipMalloc(&c, nch * 16));
  CK(hipMemset(f, 0, nch * 16));
  CK(hipMemset(b, 0, nch * 16));
  CK(hipMemset(c, 0, nch * 16));
  unsigned long long* ctr;
  CK(hipMalloc(&ctr, 16));
  CK(hipMemset(ctr, 0, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double S = (double)nch * 16;
  Run r{};
  r.f = f;
  r.b = b;
  r.n = nch;
  // references
  r.mode = 0;
  r.f = f;
  r.b = c;
  r.grid = cus * 32;
  printf("copy                          %7.3f ms  %6.2f TB/s\n", timeit(e0, e1, launch, &r, 5),
         2 * S / timeit(e0, e1, launch, &r, 5) / 1e9);
  r.b = b;
  for (int ns = 1; ns <= 2; ++ns)
    for (int u : {4, 8}) {
      r.mode = 1;
      r.ns = ns;
      r.u = u;
      r.grid = cus * 8;
      const float ms = timeit(e0, e1, launch, &r, 5);
      printf("stream rmw ns=%d U=%d             %7.3f ms  %6.2f TB/s\n", ns, u, ms, 2 * ns * S / ms / 1e9);
    }
  if (argc > 1 && strcmp(argv[1], "pad") == 0) {
    // two states in one allocation, b = f + S + pad: does the relative placement of the two
    // streams matter?
    vec4* base;
    const size_t maxpad = (size_t)64 << 20;
    CK(hipMalloc(&base, 2 * nch * 16 + maxpad));
    CK(hipMemset(base, 0, 2 * nch * 16 + maxpad));
    const size_t pads[] = {0, 256, 1024, 4096, 16384, 65536, 262144, (size_t)1 << 20,
                           ((size_t)1 << 21) + 4096, ((size_t)32 << 20) + 8192};
    for (size_t pad : pads) {
      r.f = base;
      r.b = base + (nch * 16 + pad) / 16;
      r.mode = 1;
      r.ns = 2;
      r.u = 8;
      r.grid = cus * 8;
      float best = 1e9f;
      for (int rep = 0; rep < 3; ++rep) best = std::min(best, timeit(e0, e1, launch, &r, 5));
      printf("stream rmw ns=2 U=8 pad %10zu B %7.3f ms  %6.2f TB/s\n", pad, best, 4 * S / best / 1e9);
    }
    r.f = f;
    r.b = b;
    return 0;
  }
  // tile patterns: rows = list of chunk bit positions (after lc)
  struct Pat {
    const char* name;
    int ns, lc;
    std::vector<uint32_t> rows;
  };
  const int cb = n - 1;  // chunk bits 0..26
  std::vector<Pat> pats = {
      {"1st lc=3 rows 3..10 (contig)", 1, 3, {3, 4, 5, 6, 7, 8, 9, 10}},
      {"1st lc=3 rows 19..26 (far)", 1, 3, {19, 20, 21, 22, 23, 24, 25, 26}},
      {"1st lc=3 rows 11..18 (mid)", 1, 3, {11, 12, 13, 14, 15, 16, 17, 18}},
      {"1st lc=3 rows spread", 1, 3, {5, 8, 11, 14, 17, 20, 23, 26}},
      {"1st lc=6 rows 21..25", 1, 6, {21, 22, 23, 24, 26}},
      {"2st lc=3 rows 3..9 (contig)", 2, 3, {3, 4, 5, 6, 7, 8, 9}},
      {"2st lc=3 rows 20..26 (far)", 2, 3, {20, 21, 22, 23, 24, 25, 26}},
      {"2st lc=3 rows 12..18 (mid)", 2, 3, {12, 13, 14, 15, 16, 17, 18}},
      {"2st lc=3 rows spread", 2, 3, {5, 9, 13, 17, 20, 23, 26}},
      {"2st lc=6 rows 22..25", 2, 6, {22, 23, 24, 26}},
  };
  (void)cb;
  for (const Pat& p : pats) {
    r.mode = 2;
    r.ns = p.ns;
    r.nt = p.ns == 1 ? 256 : 128;
    const int T = p.ns == 1 ? 11 : 10;
    r.g = geo{};
    r.g.ctr = ctr;
    r.g.lc = (uint32_t)p.lc;
    r.g.h = (uint32_t)p.rows.size();
    if ((int)(p.lc + p.rows.size()) != T) {
      printf("bad pattern %s\n", p.name);
      continue;
    }
    for (size_t k = 0; k < p.rows.size(); ++k) r.g.hb[k] = p.rows[k];
    r.g.ntiles = nch >> T;
    for (int mode = 0; mode < 4; ++mode) {
      // 0: persistent block-contiguous, 1: persistent grid-strided, 2: one tile per block,
      // 3: persistent work queue
      r.persistent = mode < 2 ? 1 : mode == 3 ? 2 : 0;
      r.g.order = mode == 1;
      int per_cu = 0;
      if (r.ns == 1)
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_tile<1, 256>, 256, 0));
      else
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_tile<2, 128>, 128, 0));
      r.grid = per_cu * cus;
      uint64_t tpb = 1;
      while (tpb * (uint64_t)r.grid < r.g.ntiles) tpb <<= 1;
      r.g.tpb = (uint32_t)tpb;
      if (mode == 0) r.grid = (int)((r.g.ntiles + tpb - 1) / tpb);
      const float ms = timeit(e0, e1, launch, &r, 5);
      printf("%-30s %s %7.3f ms  %6.2f TB/s\n", p.name,
             mode == 0 ? "pers-blk " : mode == 1 ? "pers-grid" : mode == 2 ? "per-tile " : "queue    ",
             ms, 2 * p.ns * S / ms / 1e9);
    }
  }
  return 0;
}
