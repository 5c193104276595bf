// qdc_kernels.hpp — hand-written CDNA4 (gfx950) kernels for the state-vector hot path.
//
// What the reference computes (src/primitives.cu, index rules in SURVEY.md §2.1) and how it
// is laid out here:
//
//   * A state is 2^n interleaved complex amplitudes in HBM, moved in 16-byte "chunks"
//     (global_load/store_dwordx4, nontemporal): VEC = 2 amplitudes per chunk in f32, 1 in f64.
//   * Every kernel keeps each wave instruction on one contiguous KiB (64 lanes x 16 B).  Two
//     kernel families guarantee that:
//       - DIRECT kernels, when every target qubit is either inside the chunk (f32 qubit 0) or
//         at chunk-index bit >= 6: a k-qubit gate reads its 2^k "rows" (the reference's
//         INSERT_ZERO bit insertion, primitives.cu:104-105, in chunk space) as 2^k separate
//         contiguous streams;
//       - TILE kernels, when some target sits at chunk bit 0..5 (its pair mate lives in
//         another lane of the same wave): a workgroup stages a tile of 256*K contiguous
//         chunks (plus up to two "row" bits for a far target) through LDS, applies the gate
//         on LDS, and writes the tile back.
//   * Blocks own contiguous ranges of work (block-contiguous iteration, U items in flight):
//     measured on MI355X this beats persistent grid-stride loops by 10-20 % (tools/bw_probe).
//   * Reductions (densities, gate gradients) accumulate per thread, reduce the wave with
//     64-lane butterflies and the block through LDS, and write one 16-complex partial per
//     block; a finalize kernel sums partials in a fixed order (deterministic, no atomics, no
//     host round trip per gate).
//   * The reverse sweep is fused: one pass reads fwd and bwd once, uncomputes fwd,
//     accumulates the gradient from (bwd, uncomputed fwd) and pulls bwd back — 4S bytes
//     instead of the reference's 6S with a host sync in the middle (circuit.rs:320-326).
//
// Gate matrices travel as kernel arguments (kernarg → SGPRs), never as global __constant__
// symbols, so there is no cross-thread race (README.md:13).
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace qdc {

#ifdef QDC_F64
using real = double;
typedef double vec16 __attribute__((ext_vector_type(2)));
#else
using real = float;
typedef float vec16 __attribute__((ext_vector_type(4)));
#endif

struct cx {
  real x, y;
};

constexpr int VEC = 16 / (int)sizeof(cx);  // amplitudes per 16-byte chunk: 2 (f32) / 1 (f64)
constexpr int LV = (VEC == 2) ? 1 : 0;      // log2(VEC)
constexpr int BLOCK = 256;                  // 4 waves of 64
constexpr int RED = 16;                     // complex values per reduction partial
constexpr int LOWBITS = 6;                  // chunk bits that index lanes of one wave

struct alignas(16) chunk {
  cx v[VEC];
};

template <int R>
struct mat {
  cx a[R * R];  // row-major
};
struct diag4 {
  cx a[4];
};

// nontemporal 16-byte chunk access (streams larger than every cache level)
// Every state lives in global memory: the accesses go through address space 1, so they stay
// global_load/store even where a laundered pointer (asm "+v") lost the address space
// (flat_* would also count in lgkmcnt and complete out of order).
// (QDC_NT_LOAD / QDC_NT_STORE = 0: plain accesses, for A/B builds, tools/build_variant.sh)
#ifndef QDC_NT_LOAD
#define QDC_NT_LOAD 1
#endif
#ifndef QDC_NT_STORE
#define QDC_NT_STORE 1
#endif
typedef __attribute__((address_space(1))) vec16 gvec16;
__device__ __forceinline__ chunk ldc(const chunk* p) {
#if QDC_NT_LOAD
  const vec16 v = __builtin_nontemporal_load((const gvec16*)(p));
#else
  const vec16 v = *(const gvec16*)(p);
#endif
  return __builtin_bit_cast(chunk, v);
}
__device__ __forceinline__ void stc(chunk* p, const chunk& c) {
#if QDC_NT_STORE
  __builtin_nontemporal_store(__builtin_bit_cast(vec16, c), (gvec16*)(p));
#else
  *(gvec16*)(p) = __builtin_bit_cast(vec16, c);
#endif
}

__device__ __forceinline__ cx cmul(cx a, cx b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
// c + a*b
__device__ __forceinline__ cx cfma(cx a, cx b, cx c) {
  return {fma(a.x, b.x, fma(-a.y, b.y, c.x)), fma(a.x, b.y, fma(a.y, b.x, c.y))};
}
// c + a*conj(b)
__device__ __forceinline__ cx cfma_conj(cx a, cx b, cx c) {
  return {fma(a.x, b.x, fma(a.y, b.y, c.x)), fma(a.y, b.x, fma(-a.x, b.y, c.y))};
}
__device__ __forceinline__ cx cadd(cx a, cx b) { return {a.x + b.x, a.y + b.y}; }

__device__ __forceinline__ uint64_t insert_zero(uint64_t x, uint32_t b) {
  const uint64_t low = x & ((1ull << b) - 1ull);
  return ((x - low) << 1) | low;
}

template <int R>
__device__ __forceinline__ void matvec(const mat<R>& m, cx (&x)[R]) {
  cx y[R];
#pragma unroll
  for (int p = 0; p < R; ++p) {
    cx t = cmul(m.a[p * R], x[0]);
#pragma unroll
    for (int q = 1; q < R; ++q) t = cfma(m.a[p * R + q], x[q], t);
    y[p] = t;
  }
#pragma unroll
  for (int p = 0; p < R; ++p) x[p] = y[p];
}

// Per-gate operation applied to one R-vector: the op kinds share every kernel skeleton.
enum OpKind { OP_APPLY = 0, OP_REVERSE = 1, OP_REVERSE_GRAD = 2, OP_INJECT = 3,
              OP_INJECT_FIRST = 4, OP_DENSITY = 5, OP_GRAD = 6 };

constexpr bool op_two_states(int op) { return op != OP_APPLY && op != OP_DENSITY; }
constexpr bool op_reduces(int op) { return op == OP_REVERSE_GRAD || op == OP_DENSITY || op == OP_GRAD; }
constexpr bool op_writes_f(int op) { return op == OP_APPLY || op == OP_REVERSE || op == OP_REVERSE_GRAD; }
constexpr bool op_writes_b(int op) {
  return op == OP_REVERSE || op == OP_REVERSE_GRAD || op == OP_INJECT || op == OP_INJECT_FIRST;
}
constexpr bool op_reads_b(int op) {
  return op == OP_REVERSE || op == OP_REVERSE_GRAD || op == OP_INJECT || op == OP_GRAD;
}

// The math of each op on one canonical R-vector (f = first state, b = second state).
//   APPLY:        f <- A f                                  (q1gate/q2gate, pr.cu:513-646)
//   REVERSE[_GRAD]: f <- A f; [acc[pR+q] += b[p] f[q]]; b <- B b   (circuit.rs:280-392)
//   INJECT[_FIRST]: b <- [b +] A (2 conj f)                 (circuit.rs:393-420)
//   DENSITY:      acc[pR+q] += f[p] conj(f[q])              (pr.cu:689-837)
//   GRAD:         acc[pR+q] += b[p] f[q]                    (pr.cu:202-354)
template <int OP, int R>
__device__ __forceinline__ void op_vector(const mat<R>& A, const mat<R>& B, cx (&f)[R],
                                          cx (&b)[R], cx* acc) {
  if constexpr (OP == OP_APPLY) {
    matvec<R>(A, f);
  } else if constexpr (OP == OP_REVERSE || OP == OP_REVERSE_GRAD) {
    matvec<R>(A, f);
    if constexpr (OP == OP_REVERSE_GRAD) {
#pragma unroll
      for (int p = 0; p < R; ++p)
#pragma unroll
        for (int q = 0; q < R; ++q) acc[p * R + q] = cfma(b[p], f[q], acc[p * R + q]);
    }
    matvec<R>(B, b);
  } else if constexpr (OP == OP_INJECT || OP == OP_INJECT_FIRST) {
    cx t[R];
#pragma unroll
    for (int q = 0; q < R; ++q) t[q] = {2 * f[q].x, -2 * f[q].y};
    matvec<R>(A, t);
#pragma unroll
    for (int p = 0; p < R; ++p) b[p] = (OP == OP_INJECT) ? cadd(b[p], t[p]) : t[p];
  } else if constexpr (OP == OP_DENSITY) {
#pragma unroll
    for (int p = 0; p < R; ++p)
#pragma unroll
      for (int q = 0; q < R; ++q) acc[p * R + q] = cfma_conj(f[p], f[q], acc[p * R + q]);
  } else {  // OP_GRAD
#pragma unroll
    for (int p = 0; p < R; ++p)
#pragma unroll
      for (int q = 0; q < R; ++q) acc[p * R + q] = cfma(b[p], f[q], acc[p * R + q]);
  }
}

// ---------------------------------------------------------------------------------------
// Block reduction of K complex accumulators → one RED-wide partial per block.
// ---------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ void block_reduce_store(cx (&acc)[K], cx* __restrict__ out) {
  __shared__ cx red[BLOCK / 64][K];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    real x = acc[k].x, y = acc[k].y;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      x += __shfl_xor(x, o, 64);
      y += __shfl_xor(y, o, 64);
    }
    if (lane == 0) red[wave][k] = {x, y};
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < RED) {
    cx s = {0, 0};
    if (t < K) {
      s = red[0][t];
#pragma unroll
      for (int w = 1; w < BLOCK / 64; ++w) s = cadd(s, red[w][t]);
    }
    out[t] = s;  // K < RED: the unused tail of the partial is written as zeros
  }
}

// ---------------------------------------------------------------------------------------
// DIRECT family: row layouts.  MODE 0: every target bit is a chunk-index bit >= LOWBITS
// (rows are whole chunks, each row a contiguous stream).  MODE 1: (VEC == 2) qubit 0 is a
// target and it is the row's LOW index bit (q1 target, or q2 pos1).  MODE 2: (q2) qubit 0 is
// pos2, the row's HIGH bit.  Row r of a q2 item is (P2, P1) = (r >> 1, r & 1), as in
// primitives.cu:596-597.
// ---------------------------------------------------------------------------------------
struct geo {
  uint64_t items;  // work items (one R-vector group of chunks each)
  uint64_t sa;     // chunk stride of row bit A (q1: the target; q2 MODE 0: pos2; MODE 1/2: hi)
  uint64_t sb;     // chunk stride of row bit B (q2 MODE 0: pos1)
  uint32_t lo;     // chunk bit positions for zero insertion (lower first)
  uint32_t hi;
  uint32_t it;     // items per thread (block-contiguous iteration)
  uint32_t xcd;    // 1: XCD-aware block order (the blocks one XCD runs own adjacent ranges)
  uint64_t gm;     // gap mask: chunk c of a state lives at c + (c & gm) (interleaved pair)
};

// Blocks are dispatched round-robin over the 8 XCDs (block b on XCD b % 8).  The XCD-aware
// order gives XCD x the contiguous block range [x G/8, (x+1) G/8) (G a multiple of 8, else
// the identity), so each XCD streams its own part of the state.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t grid, uint32_t on) {
  if (!on || (grid & 7u)) return b;
  return (b & 7u) * (grid >> 3) + (b >> 3);
}

template <int R, int MODE>
struct rows {
  static constexpr int NC = (MODE == 0) ? R : R / 2;  // chunks per item (per state)
  static constexpr int G = (MODE == 0) ? VEC : 1;     // independent R-vectors per item

  __device__ static __forceinline__ void chunks(const geo& g, uint64_t i, uint64_t (&c)[NC]) {
    if constexpr (R == 2 && MODE == 0) {
      c[0] = insert_zero(i, g.lo);
      c[1] = c[0] + g.sa;
    } else if constexpr (R == 2) {
      c[0] = i;
    } else if constexpr (MODE == 0) {
      const uint64_t b = insert_zero(insert_zero(i, g.lo), g.hi);
      c[0] = b;
      c[1] = b + g.sb;
      c[2] = b + g.sa;
      c[3] = b + g.sa + g.sb;
    } else {
      c[0] = insert_zero(i, g.hi);
      c[1] = c[0] + g.sa;
    }
  }
  __device__ static __forceinline__ void split(const chunk (&ch)[NC], cx (&x)[G][R]) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int r = 0; r < R; ++r) x[v][r] = ch[r].v[v];
    } else if constexpr (R == 2) {
      x[0][0] = ch[0].v[0];
      x[0][1] = ch[0].v[VEC - 1];
    } else if constexpr (MODE == 1) {  // chunk = P2, lane = P1
      x[0][0] = ch[0].v[0];
      x[0][1] = ch[0].v[VEC - 1];
      x[0][2] = ch[1].v[0];
      x[0][3] = ch[1].v[VEC - 1];
    } else {  // chunk = P1, lane = P2
      x[0][0] = ch[0].v[0];
      x[0][1] = ch[1].v[0];
      x[0][2] = ch[0].v[VEC - 1];
      x[0][3] = ch[1].v[VEC - 1];
    }
  }
  __device__ static __forceinline__ void merge(const cx (&x)[G][R], chunk (&ch)[NC]) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int r = 0; r < R; ++r) ch[r].v[v] = x[v][r];
    } else if constexpr (R == 2) {
      ch[0].v[0] = x[0][0];
      ch[0].v[VEC - 1] = x[0][1];
    } else if constexpr (MODE == 1) {
      ch[0].v[0] = x[0][0];
      ch[0].v[VEC - 1] = x[0][1];
      ch[1].v[0] = x[0][2];
      ch[1].v[VEC - 1] = x[0][3];
    } else {
      ch[0].v[0] = x[0][0];
      ch[1].v[0] = x[0][1];
      ch[0].v[VEC - 1] = x[0][2];
      ch[1].v[VEC - 1] = x[0][3];
    }
  }
};

// One kernel skeleton for every op of the direct family.  Block b owns the items
// [b*BLOCK*it, (b+1)*BLOCK*it); each step keeps U items (U*NC chunks per state) in flight.
template <int OP, int R, int MODE, int U>
__global__ __launch_bounds__(BLOCK) void k_direct(chunk* __restrict__ f, chunk* __restrict__ b,
                                                  mat<R> A, mat<R> B, geo g,
                                                  cx* __restrict__ partials) {
  using L = rows<R, MODE>;
  constexpr int NACC = op_reduces(OP) ? R * R : 1;
  cx acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = {0, 0};
  const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, g.xcd);
  const uint64_t start = (uint64_t)blk * BLOCK * g.it + threadIdx.x;
  // blocks whose items all exist (every block of a power-of-two state) run without per-item
  // guards: a guarded load is a branch the waitcnt pass drains in-flight loads around
  auto body = [&](auto guarded) __attribute__((always_inline)) {
  for (uint32_t step = 0; step < g.it; step += U) {
    uint64_t c[U][L::NC];
    chunk fc[U][L::NC], bc[U][L::NC];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = start + (uint64_t)(step + u) * BLOCK;
      ok[u] = !decltype(guarded)::value || ((step + u < g.it) && i < g.items);
      L::chunks(g, ok[u] ? i : 0, c[u]);
#pragma unroll
      for (int k = 0; k < L::NC; ++k) c[u][k] += c[u][k] & g.gm;
      if (ok[u]) {
#pragma unroll
        for (int k = 0; k < L::NC; ++k) {
          fc[u][k] = ldc(f + c[u][k]);
          if constexpr (op_reads_b(OP)) bc[u][k] = ldc(b + c[u][k]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      cx fx[L::G][R], bx[L::G][R];
      L::split(fc[u], fx);
      if constexpr (op_reads_b(OP)) L::split(bc[u], bx);
#pragma unroll
      for (int gg = 0; gg < L::G; ++gg) op_vector<OP, R>(A, B, fx[gg], bx[gg], acc);
      if constexpr (op_writes_f(OP)) {
        L::merge(fx, fc[u]);
#pragma unroll
        for (int k = 0; k < L::NC; ++k) stc(f + c[u][k], fc[u][k]);
      }
      if constexpr (op_writes_b(OP)) {
        L::merge(bx, bc[u]);
#pragma unroll
        for (int k = 0; k < L::NC; ++k) stc(b + c[u][k], bc[u][k]);
      }
    }
  }
  };
  if ((uint64_t)(blk + 1) * BLOCK * g.it <= g.items && g.it % U == 0)
    body(std::false_type{});
  else
    body(std::true_type{});
  if constexpr (op_reduces(OP)) block_reduce_store<NACC>(acc, partials + (uint64_t)blockIdx.x * RED);
}

// ---------------------------------------------------------------------------------------
// TILE family: a workgroup stages a tile of TB = BLOCK*K contiguous... chunks of each state in
// LDS.  Tile-local chunk index c (0..TB): low `l` bits contiguous in HBM, the next `h` bits
// are "row" bits placed at global chunk bits hb[0] < hb[1] (far targets).  Every wave
// instruction of the load/store moves 64 consecutive chunks (l >= 8).  The gate acts on
// tile-local amplitude bits t1 (pos1 / q1 target) and t2 (pos2).
// ---------------------------------------------------------------------------------------
struct tgeo {
  uint64_t ntiles;
  uint32_t tpb;    // tiles per block (block-contiguous)
  uint32_t l;      // contiguous low chunk bits of a tile
  uint32_t h;      // row bits (0..2)
  uint32_t hb0, hb1;  // global chunk bit of row bit 0 / 1
  uint32_t t1, t2;    // tile-local amplitude bits of the gate's index bits 0 (pos1) and 1 (pos2)
  uint32_t xcd;       // XCD-aware block order (geo::xcd)
  uint64_t gm;        // gap mask (geo::gm)
  uint32_t pf;        // the next tile's loads in flight during this tile's math (round 6)
};

__device__ __forceinline__ uint64_t tile_base(const tgeo& tg, uint64_t tile) {
  uint64_t base = tile << tg.l;
  if (tg.h > 0) base = insert_zero(base, tg.hb0);
  if (tg.h > 1) base = insert_zero(base, tg.hb1);
  return base;
}
__device__ __forceinline__ uint64_t tile_chunk(const tgeo& tg, uint64_t base, uint32_t c) {
  uint64_t g = base + (c & ((1u << tg.l) - 1u));
  if (tg.h > 0) g += (uint64_t)((c >> tg.l) & 1u) << tg.hb0;
  if (tg.h > 1) g += (uint64_t)((c >> (tg.l + 1)) & 1u) << tg.hb1;
  return g;
}

template <int OP, int R, int K>
__global__ __launch_bounds__(BLOCK) void k_tile(chunk* __restrict__ f, chunk* __restrict__ b,
                                                mat<R> A, mat<R> B, tgeo tg,
                                                cx* __restrict__ partials) {
  constexpr int TB = BLOCK * K;                 // chunks per state per tile
  constexpr int NS = op_two_states(OP) ? 2 : 1;
  __shared__ chunk lds[NS][TB];
  constexpr int NACC = op_reduces(OP) ? R * R : 1;
  cx acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = {0, 0};
  const uint32_t t = threadIdx.x;
  const uint32_t tc = 1u << (tg.l + tg.h);     // chunks per tile (== TB except tiny states)
  const uint32_t ng = (tc * VEC) / R;          // gate groups per tile
  const uint32_t lo_t = tg.t1 < tg.t2 ? tg.t1 : tg.t2;
  const uint32_t hi_t = tg.t1 < tg.t2 ? tg.t2 : tg.t1;
  const uint64_t tile0 = (uint64_t)xcd_block(blockIdx.x, gridDim.x, tg.xcd) * tg.tpb;
  // A block's tiles are software-pipelined (round 6): the next tile's loads are issued into
  // registers before this tile's gate math on LDS and its stores, so a block with several
  // tiles (the reducing launches: tpb = 16-32) keeps its loads in flight through the compute
  // phase.  (Streaming launches run one tile per block.)
  uint64_t gi[K];
  chunk rf[K], rb[K];
  auto load = [&](uint64_t tile) __attribute__((always_inline)) {
    const uint64_t base = tile_base(tg, tile);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k * BLOCK + t >= tc) break;
      uint64_t g = tile_chunk(tg, base, k * BLOCK + t);
      g += g & tg.gm;
      rf[k] = ldc(f + g);
      if constexpr (op_reads_b(OP)) rb[k] = ldc(b + g);
    }
  };
  if (tile0 < tg.ntiles) load(tile0);
  for (uint32_t tt = 0; tt < tg.tpb; ++tt) {
    const uint64_t tile = tile0 + tt;
    if (tile >= tg.ntiles) break;
    {
      const uint64_t base = tile_base(tg, tile);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (k * BLOCK + t >= tc) break;
        gi[k] = tile_chunk(tg, base, k * BLOCK + t);
        gi[k] += gi[k] & tg.gm;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k * BLOCK + t >= tc) break;
      lds[0][k * BLOCK + t] = rf[k];
      if constexpr (op_reads_b(OP)) lds[NS - 1][k * BLOCK + t] = rb[k];
    }
    __syncthreads();
    if (tg.pf && tt + 1 < tg.tpb && tile + 1 < tg.ntiles) load(tile + 1);
    cx* lf = reinterpret_cast<cx*>(&lds[0][0]);
    cx* lb = reinterpret_cast<cx*>(&lds[NS - 1][0]);
    for (uint32_t grp = t; grp < ng; grp += BLOCK) {
      uint32_t a0;
      uint32_t off[R];
      if constexpr (R == 2) {
        a0 = (uint32_t)insert_zero(grp, tg.t1);
        off[0] = 0;
        off[1] = 1u << tg.t1;
      } else {
        a0 = (uint32_t)insert_zero(insert_zero(grp, lo_t), hi_t);
        off[0] = 0;
        off[1] = 1u << tg.t1;
        off[2] = 1u << tg.t2;
        off[3] = off[1] + off[2];
      }
      cx fx[R], bx[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        fx[r] = lf[a0 + off[r]];
        if constexpr (op_reads_b(OP)) bx[r] = lb[a0 + off[r]];
      }
      op_vector<OP, R>(A, B, fx, bx, acc);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (op_writes_f(OP)) lf[a0 + off[r]] = fx[r];
        if constexpr (op_writes_b(OP)) lb[a0 + off[r]] = bx[r];
      }
    }
    if constexpr (op_writes_f(OP) || op_writes_b(OP)) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (k * BLOCK + t >= tc) break;
        if constexpr (op_writes_f(OP)) stc(f + gi[k], lds[0][k * BLOCK + t]);
        if constexpr (op_writes_b(OP)) stc(b + gi[k], lds[NS - 1][k * BLOCK + t]);
      }
    }
    __syncthreads();  // the next tile overwrites lds
    if (!tg.pf && tt + 1 < tg.tpb && tile + 1 < tg.ntiles) load(tile + 1);
  }
  if constexpr (op_reduces(OP)) block_reduce_store<NACC>(acc, partials + (uint64_t)blockIdx.x * RED);
}

// ---------------------------------------------------------------------------------------
// LANE family (round 5): one 16-byte chunk per lane and state, the gate's partner
// amplitudes fetched from other lanes of the wave.  A wave's "unit" is 64 chunks: its lanes
// take the contiguous chunk bits 0..nlow-1 and the far targets' chunk bits as their top lane
// bits (a q1 at chunk bit 20: lanes 0..31 read 32 consecutive chunks of row 0, lanes 32..63
// the same chunks of row 1; targets below 6 - #far stay at their own lane bit).  Gate index
// bit k (0: pos1 / the q1 target, 1: pos2) is either a lane bit (xor mask m_k, the partner
// fetched with ds_bpermute) or, f32 only, the amplitude bit inside the chunk (qubit 0: AMPK).
// Each lane computes the rows it holds, so the op's arithmetic is the minimum R complex MACs
// per amplitude and matrix; the row a lane holds (rr) depends on its lane bits, so its
// matrix coefficients are selected once per thread.  Measured motive (tools/r5/
// stream_probe.hip): one chunk per lane in flight streams at 83-88 % of HBM, the direct rows'
// R chunks per lane at 69-74 %.
// ---------------------------------------------------------------------------------------
struct lgeo {
  uint64_t units;  // 64-chunk units of the state
  uint32_t it;     // units per wave (block-contiguous iteration; reductions)
  uint32_t nlow;   // contiguous low chunk bits of a unit (6 - nf)
  uint32_t nf;     // far targets (0..2), lane bits nlow .. 5
  uint32_t f0, f1; // their chunk bits, ascending
  uint32_t m0, m1; // lane xor masks of gate bit 0 / 1 (0 for the in-chunk bit)
  uint32_t xcd;    // XCD-aware block order (geo::xcd)
  uint64_t gm;     // gap mask (geo::gm)
};

__device__ __forceinline__ uint64_t lane_chunk(const lgeo& g, uint64_t unit, uint32_t lane) {
  uint64_t x = unit << g.nlow;
  if (g.nf > 0) x = insert_zero(x, g.f0);
  if (g.nf > 1) x = insert_zero(x, g.f1);
  x |= lane & ((1u << g.nlow) - 1u);
  if (g.nf > 0) x |= (uint64_t)((lane >> g.nlow) & 1u) << g.f0;
  if (g.nf > 1) x |= (uint64_t)((lane >> (g.nlow + 1)) & 1u) << g.f1;
  return x + (x & g.gm);
}

__device__ __forceinline__ real lane_xor(real v, uint32_t m) { return __shfl_xor(v, (int)m, 64); }
__device__ __forceinline__ chunk chunk_xor(const chunk& c, uint32_t m) {
  chunk r;
#pragma unroll
  for (int v = 0; v < VEC; ++v) r.v[v] = {lane_xor(c.v[v].x, m), lane_xor(c.v[v].y, m)};
  return r;
}

// the chunks a lane needs: P[dl] = the chunk of lane ^ mask(dl), dl over the lane bits of d
template <int R, int AMPK>
struct lane_rows {
  static constexpr uint32_t AMASK = AMPK >= 0 ? (1u << AMPK) : 0u;  // gate bit held in-chunk
  static constexpr int NP = (R == 2) ? (AMPK >= 0 ? 1 : 2) : (AMPK >= 0 ? 2 : 4);
  // P index of the lane part of a relative offset d
  __device__ static constexpr int pidx(int d) {
    const int dl = d & ~(int)AMASK;
    if constexpr (R == 4 && AMPK == 0) return dl >> 1;
    if constexpr (R == 4 && AMPK == 1) return dl;
    return dl;
  }
  // xch(x, m): the chunk x of lane (thread) ^ m
  template <class X>
  __device__ static __forceinline__ void gather(const chunk& x, uint32_t m0, uint32_t m1, chunk (&P)[NP],
                                                X&& xch) {
    P[0] = x;
    if constexpr (R == 2 && AMPK < 0) {
      P[1] = xch(x, m0);
    } else if constexpr (R == 4 && AMPK == 0) {
      P[1] = xch(x, m1);
    } else if constexpr (R == 4 && AMPK == 1) {
      P[1] = xch(x, m0);
    } else if constexpr (R == 4) {
      P[1] = xch(x, m0);
      P[2] = xch(x, m1);
      P[3] = xch(x, m0 | m1);
    }
  }
  __device__ static __forceinline__ void gather(const chunk& x, uint32_t m0, uint32_t m1, chunk (&P)[NP]) {
    gather(x, m0, m1, P, [](const chunk& c, uint32_t m) { return chunk_xor(c, m); });
  }
  // out.v[v] = sum_d cf[v][d] * (amplitude at offset d from v's row)
  __device__ static __forceinline__ void rows_out(const cx (&cf)[VEC][R], const chunk (&P)[NP], chunk& out) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      cx y = cmul(cf[v][0], at(P, v, 0));
#pragma unroll
      for (int d = 1; d < R; ++d) y = cfma(cf[v][d], at(P, v, d), y);
      out.v[v] = y;
    }
  }
  // the amplitude at relative row offset d from amplitude v's own row
  __device__ static __forceinline__ cx at(const chunk (&P)[NP], int v, int d) {
    const int vf = AMPK >= 0 ? (v ^ ((d >> (AMPK < 0 ? 0 : AMPK)) & 1)) : v;
    return P[pidx(d)].v[vf];
  }
  // own row of amplitude v: the lane bits' part rl (runtime) and the in-chunk bit (v)
  __device__ static constexpr uint32_t amp_part(int v) { return AMPK >= 0 ? ((uint32_t)v << AMPK) : 0u; }
};

// coefficient M[rr][rr ^ d] for rr = rl | amp_part(v), selected over the lane part rl
template <int R, int AMPK>
__device__ __forceinline__ cx lane_coef(const mat<R>& M, uint32_t rl, int v, int d) {
  using L = lane_rows<R, AMPK>;
  const uint32_t av = L::amp_part(v);
  cx c = M.a[av * R + (av ^ (uint32_t)d)];
#pragma unroll
  for (uint32_t r = 1; r < (uint32_t)R; ++r) {
    if (r & L::AMASK) continue;
    const uint32_t rr = r | av;
    const cx cr = M.a[rr * R + (rr ^ (uint32_t)d)];
    c.x = (rl == r) ? cr.x : c.x;
    c.y = (rl == r) ? cr.y : c.y;
  }
  return c;
}

template <int OP, int R, int AMPK, int U>
__global__ __launch_bounds__(BLOCK) void k_lane(chunk* __restrict__ f, chunk* __restrict__ b,
                                                mat<R> A, mat<R> B, lgeo g,
                                                cx* __restrict__ partials) {
  using L = lane_rows<R, AMPK>;
  constexpr int NP = L::NP;
  constexpr bool RD = op_reduces(OP);
  // accumulators per relative offset, and per in-chunk amplitude when that bit is a gate bit
  // (else both amplitudes of a chunk share the row and one accumulator set)
  constexpr int NV = AMPK >= 0 ? VEC : 1;
  constexpr int NACC = RD ? NV * R : 1;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the lane part of this lane's row index
  uint32_t rl = 0;
  if (AMPK != 0) rl |= (lane & g.m0) ? 1u : 0u;
  if (R == 4 && AMPK != 1) rl |= (lane & g.m1) ? 2u : 0u;
  // coefficients of the matrices this op applies, per own amplitude and relative offset
  constexpr bool USE_A = OP == OP_APPLY || OP == OP_REVERSE || OP == OP_REVERSE_GRAD ||
                         OP == OP_INJECT || OP == OP_INJECT_FIRST;
  constexpr bool USE_B = OP == OP_REVERSE || OP == OP_REVERSE_GRAD;
  cx ca[USE_A ? VEC : 1][R], cb[USE_B ? VEC : 1][R];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int d = 0; d < R; ++d) {
      if constexpr (USE_A) ca[v][d] = lane_coef<R, AMPK>(A, rl, v, d);
      if constexpr (USE_B) cb[v][d] = lane_coef<R, AMPK>(B, rl, v, d);
    }
  cx acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = {0, 0};
  const uint64_t blk = xcd_block(blockIdx.x, gridDim.x, g.xcd);
  // U units per wave in flight: every load of a step is issued before its first exchange;
  // a block's step covers 4U consecutive units.  Blocks whose units all exist run unguarded.
  auto body = [&](auto guarded) __attribute__((always_inline)) {
  for (uint32_t s = 0; s < g.it; s += U) {
    uint64_t cc[U];
    chunk fxs[U], bxs[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t unit = (blk * g.it + s + u) * (BLOCK / 64) + wave;
      ok[u] = !decltype(guarded)::value || unit < g.units;  // wave-uniform
      cc[u] = lane_chunk(g, ok[u] ? unit : 0, lane);
      if (ok[u]) {
        fxs[u] = ldc(f + cc[u]);
        if constexpr (op_reads_b(OP)) bxs[u] = ldc(b + cc[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const uint64_t c = cc[u];
      chunk fx = fxs[u], bx = bxs[u];
      if constexpr (OP == OP_APPLY) {
        chunk P[NP];
        L::gather(fx, g.m0, g.m1, P);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          cx y = cmul(ca[v][0], L::at(P, v, 0));
#pragma unroll
          for (int d = 1; d < R; ++d) y = cfma(ca[v][d], L::at(P, v, d), y);
          fx.v[v] = y;
        }
        stc(f + c, fx);
      } else if constexpr (OP == OP_REVERSE || OP == OP_REVERSE_GRAD) {
        chunk P[NP], Q[NP];
        L::gather(fx, g.m0, g.m1, P);
        L::gather(bx, g.m0, g.m1, Q);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          cx y = cmul(ca[v][0], L::at(P, v, 0));
#pragma unroll
          for (int d = 1; d < R; ++d) y = cfma(ca[v][d], L::at(P, v, d), y);
          fx.v[v] = y;  // uncomputed own amplitude
          if constexpr (OP == OP_REVERSE_GRAD) {
#pragma unroll
            for (int d = 0; d < R; ++d)
              acc[(AMPK >= 0 ? v : 0) * R + d] = cfma(L::at(Q, v, d), y, acc[(AMPK >= 0 ? v : 0) * R + d]);
          }
          cx z = cmul(cb[v][0], L::at(Q, v, 0));
#pragma unroll
          for (int d = 1; d < R; ++d) z = cfma(cb[v][d], L::at(Q, v, d), z);
          bx.v[v] = z;
        }
        stc(f + c, fx);
        stc(b + c, bx);
      } else if constexpr (OP == OP_INJECT || OP == OP_INJECT_FIRST) {
        chunk t;
#pragma unroll
        for (int v = 0; v < VEC; ++v) t.v[v] = {2 * fx.v[v].x, -2 * fx.v[v].y};
        chunk P[NP];
        L::gather(t, g.m0, g.m1, P);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          cx y = cmul(ca[v][0], L::at(P, v, 0));
#pragma unroll
          for (int d = 1; d < R; ++d) y = cfma(ca[v][d], L::at(P, v, d), y);
          bx.v[v] = (OP == OP_INJECT) ? cadd(bx.v[v], y) : y;
        }
        stc(b + c, bx);
      } else if constexpr (OP == OP_DENSITY) {
        chunk P[NP];
        L::gather(fx, g.m0, g.m1, P);
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
          for (int d = 0; d < R; ++d) acc[(AMPK >= 0 ? v : 0) * R + d] =
              cfma_conj(fx.v[v], L::at(P, v, d), acc[(AMPK >= 0 ? v : 0) * R + d]);
      } else {  // OP_GRAD
        chunk P[NP];
        L::gather(fx, g.m0, g.m1, P);
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
          for (int d = 0; d < R; ++d) acc[(AMPK >= 0 ? v : 0) * R + d] =
              cfma(bx.v[v], L::at(P, v, d), acc[(AMPK >= 0 ? v : 0) * R + d]);
      }
    }
  }
  };
  if ((blk + 1) * g.it * (BLOCK / 64) <= g.units)
    body(std::false_type{});
  else
    body(std::true_type{});
  if constexpr (RD) {
    // sum over the lanes that share a row index (the lane bits outside the gate's masks),
    // then one lane per row class stores its VEC*R sums at their absolute (p, q) slots
    __shared__ cx red[BLOCK / 64][R * R];
    const uint32_t tm = g.m0 | g.m1;
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      real x = acc[k].x, y = acc[k].y;
#pragma unroll
      for (uint32_t o = 32; o > 0; o >>= 1) {
        if (tm & o) continue;  // uniform
        x += __shfl_xor(x, (int)o, 64);
        y += __shfl_xor(y, (int)o, 64);
      }
      acc[k] = {x, y};
    }
    if ((lane & ~tm) == 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const uint32_t rr = rl | L::amp_part(v);
#pragma unroll
        for (int d = 0; d < R; ++d) {
          // REVERSE_GRAD: p from b (offset), q = own uncomputed f; others: p own, q offset
          const uint32_t idx = (OP == OP_REVERSE_GRAD) ? ((rr ^ (uint32_t)d) * R + rr)
                                                       : (rr * R + (rr ^ (uint32_t)d));
          red[wave][idx] = acc[v * R + d];
        }
      }
    }
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < RED) {
      cx s = {0, 0};
      if (t < R * R) {
        s = red[0][t];
#pragma unroll
        for (int w = 1; w < BLOCK / 64; ++w) s = cadd(s, red[w][t]);
      }
      partials[(uint64_t)blockIdx.x * RED + t] = s;
    }
  }
}

// Block-wide LANE variant for streaming one-state ops and injections (QDC_LANE_BLK): a unit is
// 1024 chunks, one per thread of a 1024-thread block; far targets take the top thread bits, so
// every wave instruction moves one contiguous KiB and a block reads runs of 1024 / R chunks of
// each row; partners come through LDS (16 KiB, one barrier).  Measured motive (tools/r5/
// stream_probe2.hip): at far row bits where the DRAM mapping makes two 512-B streams per wave
// slow (row bit 20: 72.6 %), 8 KiB runs per row and block stream at 77 %.
constexpr int LB_NT = 1024;
template <int OP, int R, int AMPK>
__global__ __launch_bounds__(LB_NT) void k_lane_blk(chunk* __restrict__ f, chunk* __restrict__ b,
                                                    mat<R> A, lgeo g) {
  static_assert(OP == OP_APPLY || OP == OP_INJECT || OP == OP_INJECT_FIRST, "streaming ops");
  using L = lane_rows<R, AMPK>;
  __shared__ chunk lds[LB_NT];
  const uint32_t t = threadIdx.x;
  uint32_t rl = 0;
  if (AMPK != 0) rl |= (t & g.m0) ? 1u : 0u;
  if (R == 4 && AMPK != 1) rl |= (t & g.m1) ? 2u : 0u;
  cx ca[VEC][R];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int d = 0; d < R; ++d) ca[v][d] = lane_coef<R, AMPK>(A, rl, v, d);
  const uint64_t unit = xcd_block(blockIdx.x, gridDim.x, g.xcd);
  const uint64_t c = lane_chunk(g, unit, t);
  chunk x = ldc(f + c), bx;
  if constexpr (OP == OP_INJECT) bx = ldc(b + c);
  if constexpr (OP != OP_APPLY) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) x.v[v] = {2 * x.v[v].x, -2 * x.v[v].y};
  }
  lds[t] = x;
  __syncthreads();
  chunk P[L::NP], y;
  L::gather(x, g.m0, g.m1, P, [&](const chunk&, uint32_t m) { return lds[t ^ m]; });
  L::rows_out(ca, P, y);
  if constexpr (OP == OP_APPLY) {
    stc(f + c, y);
  } else {
    if constexpr (OP == OP_INJECT) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) y.v[v] = cadd(bx.v[v], y.v[v]);
    }
    stc(b + c, y);
  }
}

// ---------------------------------------------------------------------------------------
// Diagonal two-qubit gates: purely elementwise over chunks, every position pair is a fully
// contiguous stream.  k = 2 bit(i,pos2) + bit(i,pos1)  (primitives.cu:649-672, 398-452).
//   DIAG_APPLY: s <- d s;  DIAG_REVERSE[_GRAD]: f <- dc f; [G[k] += b f]; b <- d b;
//   DIAG_GRAD: G[k] += b f.
// ---------------------------------------------------------------------------------------
enum DiagOp { DIAG_APPLY = 0, DIAG_REVERSE = 1, DIAG_REVERSE_GRAD = 2, DIAG_GRAD = 3 };

__device__ __forceinline__ cx pick4(const diag4& d, uint32_t k) {
  const cx lo = (k & 1) ? d.a[1] : d.a[0];
  const cx hi = (k & 1) ? d.a[3] : d.a[2];
  return (k & 2) ? hi : lo;
}

struct dgeo {
  uint64_t nchunks;
  uint32_t it;
  uint32_t p2, p1;
  uint64_t gm;  // gap mask (geo::gm)
  uint32_t xcd;  // XCD-aware block order (the blocks of one XCD own adjacent ranges)
};

template <int OP, int U>
__global__ __launch_bounds__(BLOCK) void k_diag(chunk* __restrict__ f, chunk* __restrict__ b,
                                                diag4 dc, diag4 d, dgeo g,
                                                cx* __restrict__ partials) {
  constexpr bool RED_ = (OP == DIAG_REVERSE_GRAD || OP == DIAG_GRAD);
  constexpr bool TWO = (OP != DIAG_APPLY);
  cx acc[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
  const uint32_t blk = xcd_block(blockIdx.x, gridDim.x, g.xcd);
  const uint64_t start = (uint64_t)blk * BLOCK * g.it + threadIdx.x;
  auto body = [&](auto guarded) __attribute__((always_inline)) {  // as k_direct
  for (uint32_t step = 0; step < g.it; step += U) {
    chunk fc[U], bc[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = start + (uint64_t)(step + u) * BLOCK;
      ok[u] = !decltype(guarded)::value || ((step + u < g.it) && i < g.nchunks);
      if (ok[u]) {
        fc[u] = ldc(f + (i + (i & g.gm)));
        if constexpr (TWO) bc[u] = ldc(b + (i + (i & g.gm)));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const uint64_t i = start + (uint64_t)(step + u) * BLOCK;
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const uint64_t a = i * VEC + v;
        const uint32_t k = (uint32_t)(((a >> g.p2) & 1) << 1 | ((a >> g.p1) & 1));
        if constexpr (OP == DIAG_APPLY) {
          fc[u].v[v] = cmul(pick4(d, k), fc[u].v[v]);
        } else if constexpr (OP == DIAG_GRAD) {
          const cx prod = cmul(bc[u].v[v], fc[u].v[v]);
#pragma unroll
          for (uint32_t kk = 0; kk < 4; ++kk) acc[kk] = cadd(acc[kk], (k == kk) ? prod : cx{0, 0});
        } else {
          const cx fv = cmul(pick4(dc, k), fc[u].v[v]);
          if constexpr (OP == DIAG_REVERSE_GRAD) {
            const cx prod = cmul(bc[u].v[v], fv);
#pragma unroll
            for (uint32_t kk = 0; kk < 4; ++kk)
              acc[kk] = cadd(acc[kk], (k == kk) ? prod : cx{0, 0});
          }
          fc[u].v[v] = fv;
          bc[u].v[v] = cmul(pick4(d, k), bc[u].v[v]);
        }
      }
      if constexpr (OP != DIAG_GRAD) stc(f + (i + (i & g.gm)), fc[u]);
      if constexpr (OP == DIAG_REVERSE || OP == DIAG_REVERSE_GRAD) stc(b + (i + (i & g.gm)), bc[u]);
    }
  }
  };
  if ((uint64_t)(blk + 1) * BLOCK * g.it <= g.nchunks && g.it % U == 0)
    body(std::false_type{});
  else
    body(std::true_type{});
  if constexpr (RED_) block_reduce_store<4>(acc, partials + (uint64_t)blockIdx.x * RED);
}

// Diagonal two-qubit gates with the diagonal index k fixed per thread and amplitude slot
// (round 6; knob QDC_DIAG_Q).  A gate position is the in-chunk amplitude bit (f32 qubit 0), a
// "thread" chunk bit (< 8: the thread index supplies it) or a "block" chunk bit (>= 8).  Blocks
// walk the state by quadrant: the block bits of chunk i are the top bits of the iteration index
// j, so every block sees one value of them and chunk i = D(j - t) + t with D the bit deposit
// (uniform).  k, the two matrix entries and the accumulator of each amplitude slot are then
// constants of the thread — per amplitude the pass costs its three complex multiplies and
// nothing else (k_diag selects entries and accumulators per amplitude).  Runs of >= 256
// contiguous chunks, as k_diag.  Host: diag_q_geo (qdc_device.hpp).  Measured at n = 28 f32
// (profiles/r6/r6k, r6l): reverse_q2_diag 73.1 % (k_diag) -> 75.4 % at 8 chunks in flight per
// state, 76.7 % at 16, 77.3 % at 16 with 4096 blocks (the default).
struct dqgeo {
  uint64_t gm;        // gap mask (geo::gm)
  uint32_t it;        // chunks per thread (a multiple of U)
  uint32_t qshift;    // j bit where the quadrant index starts (log2 nchunks - nb)
  uint32_t c0, c1;    // block chunk bits, ascending (nb of them are valid)
  uint32_t nb;        // 0, 1 or 2
  // where the k bit of pos1 / pos2 comes from: 0x100 the amplitude slot v, 0x200 | s thread
  // bit s, 0x400 | q bit q of the block's quadrant index
  uint32_t k1, k2;
};

template <int OP, int U>
__global__ __launch_bounds__(BLOCK) void k_diag_q(chunk* __restrict__ f, chunk* __restrict__ b,
                                                  diag4 dc, diag4 d, dqgeo g,
                                                  cx* __restrict__ partials) {
  constexpr bool RED_ = (OP == DIAG_REVERSE_GRAD || OP == DIAG_GRAD);
  constexpr bool TWO = (OP != DIAG_APPLY);
  const uint32_t t = threadIdx.x;
  const uint64_t jb = (uint64_t)blockIdx.x * BLOCK * g.it;
  const uint32_t qd = (uint32_t)(jb >> g.qshift);  // this block's quadrant
  uint32_t k[VEC];  // k = 2 bit(pos2) + bit(pos1) per amplitude slot
  auto kbit = [&](uint32_t enc, int v) -> uint32_t {
    if (enc & 0x100u) return (uint32_t)v & 1u;
    if (enc & 0x200u) return (t >> (enc & 0xffu)) & 1u;
    return (qd >> (enc & 0xffu)) & 1u;
  };
#pragma unroll
  for (int v = 0; v < VEC; ++v) k[v] = (kbit(g.k2, v) << 1) | kbit(g.k1, v);
  cx ca[VEC], cb[VEC], acc[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    ca[v] = pick4(OP == DIAG_APPLY ? d : dc, k[v]);
    cb[v] = pick4(d, k[v]);
    acc[v] = {0, 0};
  }
  // D(j - t): the block bits deposited at c0 (< c1), from the quadrant index
  const uint64_t jmask = ((uint64_t)1 << g.qshift) - 1;
  auto deposit = [&](uint64_t j) -> uint64_t {
    uint64_t x = j & jmask;
    if (g.nb >= 1) x = insert_zero(x, g.c0) | ((uint64_t)(qd & 1u) << g.c0);
    if (g.nb >= 2) x = insert_zero(x, g.c1) | ((uint64_t)((qd >> 1) & 1u) << g.c1);
    return x;
  };
  for (uint32_t step = 0; step < g.it; step += U) {
    chunk fc[U], bc[U];
    uint64_t a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = deposit(jb + (uint64_t)(step + u) * BLOCK) + t;
      a[u] = i + (i & g.gm);
      fc[u] = ldc(f + a[u]);
      if constexpr (TWO) bc[u] = ldc(b + a[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        if constexpr (OP == DIAG_APPLY) {
          fc[u].v[v] = cmul(ca[v], fc[u].v[v]);
        } else if constexpr (OP == DIAG_GRAD) {
          acc[v] = cfma(bc[u].v[v], fc[u].v[v], acc[v]);
        } else {
          const cx fv = cmul(ca[v], fc[u].v[v]);
          if constexpr (OP == DIAG_REVERSE_GRAD) acc[v] = cfma(bc[u].v[v], fv, acc[v]);
          fc[u].v[v] = fv;
          bc[u].v[v] = cmul(cb[v], bc[u].v[v]);
        }
      }
      if constexpr (OP != DIAG_GRAD) stc(f + a[u], fc[u]);
      if constexpr (OP == DIAG_REVERSE || OP == DIAG_REVERSE_GRAD) stc(b + a[u], bc[u]);
    }
  }
  if constexpr (RED_) {
    cx acc4[4];
#pragma unroll
    for (uint32_t kk = 0; kk < 4; ++kk) {
      acc4[kk] = {0, 0};
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc4[kk] = cadd(acc4[kk], (k[v] == kk) ? acc[v] : cx{0, 0});
    }
    block_reduce_store<4>(acc4, partials + (uint64_t)blockIdx.x * RED);
  }
}

// ---------------------------------------------------------------------------------------
// Partial-sum finalize: one block per pending reduction slot, fixed summation order.
// dst[slot_dst[s]*RED + k] (+)= sum_b partials[s][b][k].
// ---------------------------------------------------------------------------------------
constexpr int FIN_MAX = 32;
struct fin_table {  // each slot's destination (its reduction base + slot index, resolved)
  cx* dst[FIN_MAX];
};

// Granule partials of a dynamic-tail pass, pre-summed: block (slot y, chunk x) adds the BLOCK
// partials x*BLOCK .. of slot y by a fixed tree (block_reduce_store) into one chunk partial.
#ifndef QDC_SPEC_TU  // (not in the specialized kernels' translation units)
__global__ __launch_bounds__(BLOCK) void k_dsum(const cx* __restrict__ parts, uint64_t stride,
                                                uint32_t n, cx* __restrict__ out,
                                                uint64_t out_stride) {
  const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const cx* p = parts + (uint64_t)blockIdx.y * stride + g * RED;
  cx acc[RED];
#pragma unroll
  for (int k = 0; k < RED; ++k) acc[k] = g < n ? p[k] : cx{0, 0};
  block_reduce_store<RED>(acc, out + (uint64_t)blockIdx.y * out_stride + (uint64_t)blockIdx.x * RED);
}
#endif  // QDC_SPEC_TU

// one slot per block: the sum of its nblocks block partials, then of its n2 granule partials
// (dynamic-tail passes, fgeo::dpart) — a fixed order, so the result is deterministic
#ifndef QDC_SPEC_TU  // (not in the specialized kernels' translation units)
__global__ __launch_bounds__(BLOCK) void k_finalize(const cx* __restrict__ partials,
                                                    uint64_t slot_stride, uint32_t nblocks,
                                                    fin_table tab, int accumulate, const cx* __restrict__ partials2,
                                                    uint64_t slot_stride2, uint32_t n2) {
  const cx* p = partials + (uint64_t)blockIdx.x * slot_stride;
  const cx* p2 = partials2 + (uint64_t)blockIdx.x * slot_stride2;
  cx acc[RED];
#pragma unroll
  for (int k = 0; k < RED; ++k) acc[k] = {0, 0};
  for (uint32_t blk = threadIdx.x; blk < nblocks + n2; blk += BLOCK) {
    const cx* q = blk < nblocks ? p + (uint64_t)blk * RED : p2 + (uint64_t)(blk - nblocks) * RED;
#pragma unroll
    for (int k = 0; k < RED; ++k) acc[k] = cadd(acc[k], q[k]);
  }
  __shared__ cx out[RED];
  block_reduce_store<RED>(acc, out);
  __syncthreads();
  if (threadIdx.x < RED) {
    cx* d = tab.dst[blockIdx.x] + threadIdx.x;
    *d = accumulate ? cadd(*d, out[threadIdx.x]) : out[threadIdx.x];
  }
}
#endif  // QDC_SPEC_TU


// ---------------------------------------------------------------------------------------
// FUSED family: a pass of gates whose qubits all fit one tile is
// applied in ONE HBM pass.  A tile = TB chunks of each state: `lc` contiguous low chunk bits
// (>= 3: 128-B rows) plus `h` row bits at far chunk positions hb[].  The pass runs its ops on
// LDS with a barrier between ops; each op is a register STAGE (qdc_stage.hpp): a run of gates
// within one qubit pair, applied as the host-formed products A (fwd) and B (bwd pull-back).  A
// two-state (reverse) program also accumulates the stage's Gamma = sum b0 f0^T of the
// stage-entry states, from which the host derives every gate's gradient exactly.
// Gamma: per thread in registers during an op, then a reduce-scatter over the wave
// (permlane swaps + DPP, ~V instructions for V values) and one LDS add per value into the
// wave's accumulator slot; one partial per block and gradient stage at the end.
// ---------------------------------------------------------------------------------------
#ifndef QDC_FMAX_OPS
#define QDC_FMAX_OPS 32
#endif
constexpr int FMAX_OPS = QDC_FMAX_OPS;   // gates per fused pass (>= its stages)
constexpr int FMAX_GRAD = 16;  // gradient gates per fused pass (>= its gradient stages)
#ifndef QDC_FMAX_GRAD_RQ
#define QDC_FMAX_GRAD_RQ 16
#endif
// the same for register-resident two-state passes (per-wave LDS accumulators).  Measured at
// C2 n=28: 24 / 32 give 20 % / 15 % fewer reverse passes, each 33 % / 23 % slower (more
// relayouts per stage, 7 / 6 blocks per CU): 16 is best.
constexpr int FMAX_GRAD_RQ = QDC_FMAX_GRAD_RQ;
static_assert(FMAX_GRAD_RQ >= 1 && FMAX_GRAD >= 1, "at least one reduction accumulator");
static_assert(FMAX_OPS <= 64, "rq_plan keeps stage sets in 64-bit masks");
constexpr int FMAX_ROWS = 8;   // far qubits per tile
constexpr int FACC = 32;       // reals per gradient accumulator (16 complex)

struct fop {
  uint32_t kind;  // 0: one-qubit dense, 1: two-qubit dense, 2: two-qubit diagonal; +4: gradient
  uint32_t t1;    // tile-local amplitude bit of pos1 (one-qubit: the target)
  uint32_t t2;    // tile-local amplitude bit of pos2
  uint32_t mat;   // offset (complex) of A in the matrix buffer; B follows (R^2, or 4 for diag)
};

struct fgeo {
  uint64_t ntiles;
  uint32_t tpb;    // tiles per block (block-contiguous)
  uint32_t lc;     // contiguous chunk bits
  uint32_t h;      // row bits
  uint32_t hb[FMAX_ROWS];
  uint32_t nops;
  uint32_t ngrad;  // reduction ops (Gamma stages, densities): partials in consecutive slots
  uint32_t order;  // register-resident passes: 0 block-contiguous tiles, 1 grid-strided
  uint64_t gm;     // gap mask (geo::gm); register-resident passes get their rqio offsets gapped
                   // on the host, so only the tile base is gapped here
  // Dynamic tail (one-wave register-resident passes, k_rw): blocks run tpb block-contiguous
  // tiles of the first nstat, then take tiles [nstat, nstat + ndyn) one at a time from eight
  // atomic counters (pool p = block % 8, the blocks of one XCD, owns ndyn / 8 of them), so a
  // wave that finished its static share early keeps its SIMD busy instead of leaving the partner
  // wave alone (SQ counters: waves lived 81 % of the reverse pass with static shares only).
  // ndyn = 0: static only.
  unsigned long long* dctr;  // 8 counters, FG_DCTR_STRIDE apart (own cache lines)
  uint64_t dbase;            // value of every counter at this launch's start (all advance alike)
  uint64_t nstat, ndyn;
  uint32_t dgran;            // tiles per grab (a granule); ndyn is a multiple of 8 dgran
  // Reductions stay deterministic: the static tiles of a block sum into its block partial; each
  // granule's Gamma sums go to its own partial, dpart[slot * dstride + granule * RED], so every
  // value is summed over the same tiles in the same order whichever wave ran them
  cx* dpart;
  uint64_t dstride;
};
constexpr int FG_DCTR_STRIDE = 32;  // 256 B between the pool counters
// dynamic tails compiled in (0: static shares only; Ctx::plan_dyn then never plans one)
#ifndef QDC_DYN_TAIL
#define QDC_DYN_TAIL 1
#endif

// The fgeo argument of the register-resident kernels (k_rq, k_rw: four pointers precede it),
// read through an opaque kernarg-segment pointer: the dynamic-tail fields are used once per
// grab, so they are loaded (s_load, scalar cache) at their uses instead of being held in SGPRs
// across the pass — held, they pushed the reverse kernel's SGPR spills from 27 to 57.
struct fg_kernargs {  // the kernels' leading parameters, as the kernarg segment lays them out
  void* f;
  void* b;
  const void* ops;
  const void* mats;
  fgeo fg;
};
constexpr size_t FG_KERNARG_OFFSET = offsetof(fg_kernargs, fg);
static_assert(FG_KERNARG_OFFSET == 32, "fgeo follows four pointers");
typedef const __attribute__((address_space(4))) fgeo* fg_kptr;
__device__ __forceinline__ fg_kptr fg_arg() {
  const __attribute__((address_space(4))) char* p =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (fg_kptr)(p + FG_KERNARG_OFFSET);
}

// next tile index of this block's pool (>= ndyn / 8: the pool is empty); one wave per block
__device__ __forceinline__ uint64_t fg_grab() {
  unsigned long long v = 0;
  if (threadIdx.x == 0) v = atomicAdd(fg_arg()->dctr + FG_DCTR_STRIDE * (blockIdx.x & 7u), 1ull);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((((uint64_t)hi) << 32) | lo) - fg_arg()->dbase;
}

// Complex multiply(-accumulate) for the fused kernels.  In f32 each is two v_pk_fma_f32 on the
// natural (re, im) register pairs, with op_sel/neg modifiers doing the broadcast and swap:
//   c += a.re * (f.re, f.im);   c += (-a.im * f.im, a.im * f.re)
// Gate-matrix entries stay as one SGPR pair each ("s"): left to itself the compiler
// materialises (a.re, a.re) and (-a.im, a.im) pairs — twice the SGPRs, which spill for a
// two-qubit reverse step (A and B = 32 entries) and are re-read every iteration.
#ifndef QDC_F64
typedef float pk2 __attribute__((ext_vector_type(2)));
// QDC_PK_ASM=1 (default): each packed FMA as one inline-asm statement.  The hazard recognizer
// pads inline asm conservatively — an s_nop 0 about every eighth packed FMA of a stage (r5:
// ~1000-1500 per two-state reverse program) — while for the same FMAs written with builtins
// (QDC_PK_ASM=0) it pads none: those fold the broadcast and swap into op_sel / op_sel_hi and the
// negation into a SALU xor on the matrix entry's SGPR pair (QDC_PK_VASM=0: per-lane operands
// too, where the (-b.im, b.im) pair costs a v_pk_add and two v_mov).  Measured same box,
// bit-identical outputs (profiles/r5/r5d_pk_forms_ab.txt, C2 n = 28): asm 4660-4668 gates/s,
// builtins for the matrix operands 4572-4585, builtins throughout 4354 — the pads cost nothing
// with two waves per SIMD (the partner wave issues in their cycles), the SALU xors and moves do.
#ifndef QDC_PK_ASM
#define QDC_PK_ASM 1
#endif
#ifndef QDC_PK_VASM  // (QDC_PK_ASM=0: per-lane operands still as asm)
#define QDC_PK_VASM 1
#endif
#if QDC_PK_ASM
// one instruction per asm statement, so the scheduler can interleave independent chains
__device__ __forceinline__ pk2 pk_re_fma(pk2 a, pk2 f, pk2 c) {  // c + a.re * (f.re, f.im)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(c) : "s"(a), "v"(f));
  return c;
}
__device__ __forceinline__ pk2 pk_im_fma(pk2 a, pk2 f, pk2 c) {  // c + (-a.im f.im, a.im f.re)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "+v"(c) : "s"(a), "v"(f));
  return c;
}
__device__ __forceinline__ pk2 pk_re_mul(pk2 a, pk2 f) {  // a.re * (f.re, f.im)
  pk2 r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "s"(a), "v"(f));
  return r;
}
#else
__device__ __forceinline__ pk2 pk_re_fma(pk2 a, pk2 f, pk2 c) {  // c + a.re * (f.re, f.im)
  return __builtin_elementwise_fma(__builtin_shufflevector(a, a, 0, 0), f, c);
}
__device__ __forceinline__ pk2 pk_im_fma(pk2 a, pk2 f, pk2 c) {  // c + (-a.im f.im, a.im f.re)
  const pk2 na = -a;
  return __builtin_elementwise_fma(__builtin_shufflevector(na, a, 1, 3),
                                   __builtin_shufflevector(f, f, 1, 0), c);
}
__device__ __forceinline__ pk2 pk_re_mul(pk2 a, pk2 f) {  // a.re * (f.re, f.im)
  return __builtin_shufflevector(a, a, 0, 0) * f;
}
#endif
#if QDC_PK_ASM || QDC_PK_VASM
// per-lane operands (Gamma accumulation): inline asm, whose neg_lo modifier is free (the
// builtins' (-b.im, b.im) pair costs a v_pk_add and two v_mov per use)
__device__ __forceinline__ pk2 vpk_re_fma(pk2 a, pk2 f, pk2 c) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(c) : "v"(a), "v"(f));
  return c;
}
__device__ __forceinline__ pk2 vpk_im_fma(pk2 a, pk2 f, pk2 c) {
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "+v"(c) : "v"(a), "v"(f));
  return c;
}
__device__ __forceinline__ pk2 vpk_re_mul(pk2 a, pk2 f) {
  pk2 r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "v"(f));
  return r;
}
#else
__device__ __forceinline__ pk2 vpk_re_fma(pk2 a, pk2 f, pk2 c) { return pk_re_fma(a, f, c); }
__device__ __forceinline__ pk2 vpk_im_fma(pk2 a, pk2 f, pk2 c) { return pk_im_fma(a, f, c); }
__device__ __forceinline__ pk2 vpk_re_mul(pk2 a, pk2 f) { return pk_re_mul(a, f); }
#endif
__device__ __forceinline__ cx ucfma(cx a, cx f, cx c) {  // c + a f, a wave-uniform
  const pk2 A = __builtin_bit_cast(pk2, a), F = __builtin_bit_cast(pk2, f);
  return __builtin_bit_cast(cx, pk_im_fma(A, F, pk_re_fma(A, F, __builtin_bit_cast(pk2, c))));
}
__device__ __forceinline__ cx ucmul(cx a, cx f) {  // a f, a wave-uniform
  const pk2 A = __builtin_bit_cast(pk2, a), F = __builtin_bit_cast(pk2, f);
  return __builtin_bit_cast(cx, pk_im_fma(A, F, pk_re_mul(A, F)));
}
__device__ __forceinline__ cx vcfma(cx a, cx f, cx c) {  // c + a f, both per lane
  const pk2 A = __builtin_bit_cast(pk2, a), F = __builtin_bit_cast(pk2, f);
  return __builtin_bit_cast(cx, vpk_im_fma(A, F, vpk_re_fma(A, F, __builtin_bit_cast(pk2, c))));
}
__device__ __forceinline__ cx vcmul(cx a, cx f) {  // a f, both per lane
  const pk2 A = __builtin_bit_cast(pk2, a), F = __builtin_bit_cast(pk2, f);
  return __builtin_bit_cast(cx, vpk_im_fma(A, F, vpk_re_mul(A, F)));
}
#else
__device__ __forceinline__ cx ucfma(cx a, cx f, cx c) { return cfma(a, f, c); }
__device__ __forceinline__ cx ucmul(cx a, cx f) { return cmul(a, f); }
__device__ __forceinline__ cx vcfma(cx a, cx f, cx c) { return cfma(a, f, c); }
__device__ __forceinline__ cx vcmul(cx a, cx f) { return cmul(a, f); }
#endif

// x <- M x with a wave-uniform M (row-major R x R)
template <int R>
__device__ __forceinline__ void umatvec(const cx* M, cx (&x)[R]) {
  cx y[R];
#pragma unroll
  for (int p = 0; p < R; ++p) {
    cx t = ucmul(M[p * R], x[0]);
#pragma unroll
    for (int q = 1; q < R; ++q) t = ucfma(M[p * R + q], x[q], t);
    y[p] = t;
  }
#pragma unroll
  for (int p = 0; p < R; ++p) x[p] = y[p];
}

// NQ independent x <- M x at once, their dependency chains interleaved op by op.  A complex MAC
// is two v_pk_fma_f32 on the same accumulator, and gfx950 wants 5 other VALU ops between a
// packed FMA and the next one reading its result: one 4x4 matvec has only 4 chains (its outputs),
// so on its own the compiler pads every round of them with an s_nop (r5: ~1500 per two-state
// reverse pass program, 14 % of its VALU issue).  R * NQ >= 8 chains need none.
template <int R, int NQ>
__device__ __forceinline__ void umatvec_n(const cx* M, cx (&x)[NQ][R]) {
#ifndef QDC_F64
  // per column q: the re halves of every chain, then the im halves (R * NQ ops apart)
  pk2 y[NQ][R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
#pragma unroll
    for (int p = 0; p < R; ++p)
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const pk2 a = __builtin_bit_cast(pk2, M[p * R + q]), f = __builtin_bit_cast(pk2, x[n][q]);
        y[n][p] = q == 0 ? pk_re_mul(a, f) : pk_re_fma(a, f, y[n][p]);
      }
#pragma unroll
    for (int p = 0; p < R; ++p)
#pragma unroll
      for (int n = 0; n < NQ; ++n)
        y[n][p] = pk_im_fma(__builtin_bit_cast(pk2, M[p * R + q]), __builtin_bit_cast(pk2, x[n][q]),
                            y[n][p]);
  }
#pragma unroll
  for (int n = 0; n < NQ; ++n)
#pragma unroll
    for (int p = 0; p < R; ++p) x[n][p] = __builtin_bit_cast(cx, y[n][p]);
#else
#pragma unroll
  for (int n = 0; n < NQ; ++n) umatvec<R>(M, x[n]);
#endif
}

// Lane select with a wave-uniform lane mask (v_cndmask): lanes set in `mask` take t.  Written
// as asm because LLVM folds `upper ? x[h + i] : x[i]` on a register array into a dynamically
// indexed array (a compare/select chain over every element: O(V^2) instructions).
__device__ __forceinline__ uint32_t lane_sel(uint32_t f, uint32_t t, uint64_t mask) {
  uint32_t r;
  asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mask));
  return r;
}
__device__ __forceinline__ float lane_sel(float f, float t, uint64_t mask) {
  return __uint_as_float(lane_sel(__float_as_uint(f), __float_as_uint(t), mask));
}
__device__ __forceinline__ double lane_sel(double f, double t, uint64_t mask) {
  const uint64_t fb = (uint64_t)__double_as_longlong(f), tb = (uint64_t)__double_as_longlong(t);
  const uint64_t lo = lane_sel((uint32_t)fb, (uint32_t)tb, mask);
  const uint64_t hi = lane_sel((uint32_t)(fb >> 32), (uint32_t)(tb >> 32), mask);
  return __longlong_as_double((long long)(lo | (hi << 32)));
}

// Cross-lane moves of one real (f64 as two dwords).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(v), CTRL,
                                                               0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// (a, b) -> (a', b') with a' = [a.lo-half | b.lo-half], b' = [a.hi-half | b.hi-half], halves of
// 32 lanes (W = 32, v_permlane32_swap) or alternating rows of 16 (W = 16, v_permlane16_swap)
template <int W>
__device__ __forceinline__ void half_swap(float& a, float& b) {
  if constexpr (W == 32) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  } else {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  }
}
template <int W>
__device__ __forceinline__ void half_swap(double& a, double& b) {
  const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
  float alo = __uint_as_float((uint32_t)ua), ahi = __uint_as_float((uint32_t)(ua >> 32));
  float blo = __uint_as_float((uint32_t)ub), bhi = __uint_as_float((uint32_t)(ub >> 32));
  half_swap<W>(alo, blo);
  half_swap<W>(ahi, bhi);
  a = __longlong_as_double((long long)(((uint64_t)__float_as_uint(ahi) << 32) | __float_as_uint(alo)));
  b = __longlong_as_double((long long)(((uint64_t)__float_as_uint(bhi) << 32) | __float_as_uint(blo)));
}

// Sum V reals over the 64 lanes (reduce-scatter): afterwards value idx(lane) sits in the lanes
// whose low (6 - log2 V) index bits are zero, and is added into acc[idx] (acc in LDS, one
// writer per index).  Offsets 32 and 16 are one v_permlane{32,16}_swap + one add per value
// pair; offsets 8, 4, 2, 1 are DPP moves (row_ror:8, row_half_mirror, quad_perm) with lane
// selects.  Partner lanes always agree on the bits above the current offset, so they hold the
// same index set; the lane with the offset bit set keeps the upper half.
// ATOMIC: several waves add into the same LDS accumulators (ds_add_f32)
// Timing-only ablation builds (tools/ablate.sh; results are wrong): QDC_RQ_ABL bit 0 no stage
// math, bit 1 no relayouts, bit 2 no Gamma, bit 3 Gamma without the wave reduction, bit 4
// relayouts without barriers, bit 5 no HBM loads/stores (k_rw; qdc_rq.hpp).
#ifndef QDC_RQ_ABL
#define QDC_RQ_ABL 0
#endif
template <int V, bool ATOMIC = false>
__device__ __forceinline__ void wave_reduce_add(real (&x)[V], real* acc) {
#if QDC_RQ_ABL & 8
  {
    real s = 0;
#pragma unroll
    for (int i = 0; i < V; ++i) s += x[i];
    acc[threadIdx.x & (V - 1)] += s;
    return;
  }
#endif
  constexpr uint64_t UPPER[6] = {0xFFFFFFFF00000000ull, 0xFFFF0000FFFF0000ull,
                                 0xFF00FF00FF00FF00ull, 0xF0F0F0F0F0F0F0F0ull,
                                 0xCCCCCCCCCCCCCCCCull, 0xAAAAAAAAAAAAAAAAull};
  constexpr int CTRL[6] = {0, 0, 0x128 /*row_ror:8*/, 0x141 /*row_half_mirror*/,
                           0x4E /*quad_perm 2,3,0,1*/, 0xB1 /*quad_perm 1,0,3,2*/};
  // opaque lane: keeps the compiler from hoisting this call's lane-derived index out of the
  // pass loop (a long-lived VGPR that spilled and was reloaded, with a vmcnt wait, per stage)
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  int idx = 0;
#pragma unroll
  for (int step = 0; step < 6; ++step) {
    const int o = 32 >> step;
    const int len = V >> step;
    if (len > 1) {
      const int half = len >> 1;
#pragma unroll
      for (int i = 0; i < half; ++i) {
        if (step <= 1) {
          if (step == 0) half_swap<32>(x[i], x[half + i]);
          else half_swap<16>(x[i], x[half + i]);
#ifndef QDC_F64
          if (i & 1) {  // f32: the adds of value pairs (i - 1, i) as one v_pk_add_f32
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 a = {x[i - 1], x[i]}, c = {x[half + i - 1], x[half + i]};
            a += c;
            x[i - 1] = a.x;
            x[i] = a.y;
          } else if (i == half - 1) {
            x[i] += x[half + i];
          }
#else
          x[i] += x[half + i];
#endif
        } else {
          const real mine = lane_sel(x[i], x[half + i], UPPER[step]);
          const real send = lane_sel(x[half + i], x[i], UPPER[step]);
          if (step == 2) x[i] = mine + dpp_mov<CTRL[2]>(send);
          if (step == 3) x[i] = mine + dpp_mov<CTRL[3]>(send);
          if (step == 4) x[i] = mine + dpp_mov<CTRL[4]>(send);
          if (step == 5) x[i] = mine + dpp_mov<CTRL[5]>(send);
        }
      }
      idx += (lane & o) ? half : 0;
    } else {
      if (step == 0) {
        real y = x[0];
        half_swap<32>(x[0], y);
        x[0] += y;
      } else if (step == 1) {
        real y = x[0];
        half_swap<16>(x[0], y);
        x[0] += y;
      } else if (step == 2) {
        x[0] += dpp_mov<CTRL[2]>(x[0]);
      } else if (step == 3) {
        x[0] += dpp_mov<CTRL[3]>(x[0]);
      } else if (step == 4) {
        x[0] += dpp_mov<CTRL[4]>(x[0]);
      } else {
        x[0] += dpp_mov<CTRL[5]>(x[0]);
      }
    }
  }
  const int spread = 64 / V;  // lanes holding the same idx
  if ((lane & (spread - 1)) == 0) {
    if constexpr (ATOMIC)
      atomicAdd(&acc[idx], x[0]);
    else
      acc[idx] += x[0];
  }
}

// LDS layout of a fused tile: XOR-swizzled so that lanes of one LDS access spread over all
// banks even when the op's target bits are the low ones.  Amplitude index i lives at
// swz(i) = i ^ (((i >> (4 + LV)) & 15) << LV)  (chunk c at c ^ ((c >> 4) & 15): chunks stay
// whole).  swz is linear over XOR, so swz(a0 | off) = swz(a0) ^ swz(off) with a uniform
// swz(off): addressing costs one XOR, like the unswizzled add.
__host__ __device__ __forceinline__ uint32_t swz(uint32_t i) {
  return i ^ (((i >> (4 + LV)) & 15u) << LV);
}
__device__ __forceinline__ uint32_t swz_chunk(uint32_t c) { return c ^ ((c >> 4) & 15u); }

// fop.kind: op kind (low 3 bits) + FOP_GAMMA
enum : uint32_t {
  FK_Q1 = 0,     // one-qubit stage: f <- A f [, b <- B b]
  FK_Q2 = 1,     // two-qubit stage
  FK_DIAG = 2,   // diagonal two-qubit stage
  FK_DENS1 = 3,  // one-qubit density: acc[2p+q] += f_p conj(f_q)        (read-only)
  FK_DENS2 = 4,  // two-qubit density: acc[4p+q] += f_p conj(f_q)        (read-only)
  FK_INJ1 = 5,   // one-qubit cotangent injection: b += M (2 conj f)     (two-state)
  FK_INJ2 = 6,   // two-qubit cotangent injection
};
constexpr uint32_t FOP_GAMMA = 8;  // stage also accumulates Gamma = sum b0 f0^T (two-state)

#ifndef QDC_FUSED_WAVES
#define QDC_FUSED_WAVES 4  // waves/SIMD the fused kernels are register-allocated for
#endif
// TWO: the pass carries fwd and bwd (reverse sweep); HASRED: the pass has reduction ops (Gamma,
// densities) and their LDS accumulators; WF: the pass changes fwd, so fwd is stored back
// (density-only and injection-only passes read it only).
// NT: threads per block (a tile of TB chunks is NT threads' work: fewer threads = more
// quartets per thread per stage, amortising the per-stage reduce and setup).
template <bool TWO, int TB, bool HASRED, bool WF, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 ? QDC_FUSED_WAVES : 2)))
void k_fused(chunk* __restrict__ f, chunk* __restrict__ b, const fop* __restrict__ ops,
             const cx* __restrict__ mats, fgeo fg, cx* __restrict__ partials,
             uint64_t slot_stride) {
  constexpr int NS = TWO ? 2 : 1;
  constexpr int CPT = TB / NT;  // chunks of each state per thread and tile
  static_assert(TB % NT == 0 && TB * VEC >= 4 * NT, "tile must cover the block");
  __shared__ chunk lds[NS][TB];
  __shared__ real accw[HASRED ? NT / 64 : 1][HASRED ? FMAX_GRAD : 1][FACC];
  const uint32_t t = threadIdx.x;
  const int wave = t >> 6;
  if constexpr (HASRED) {
    for (uint32_t i = t; i < (NT / 64) * FMAX_GRAD * FACC; i += NT)
      (&accw[0][0][0])[i] = 0;
  }
  // a tile is always TB chunks (lc + h == log2 TB; the host fuses nothing in smaller states),
  // so no per-chunk guards: divergent guards make the waitcnt pass drain every prefetch
  constexpr uint32_t ta = TB * VEC;  // amplitudes per tile
  cx* lf = reinterpret_cast<cx*>(&lds[0][0]);
  cx* lb = reinterpret_cast<cx*>(&lds[NS - 1][0]);
  // thread-owned tile chunks c = t + i*NT sit at the same offset from every tile's base
  uint64_t off[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const uint32_t c = t + (uint32_t)i * NT;
    uint64_t o = c & ((1u << fg.lc) - 1u);
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < fg.h) o += (uint64_t)((c >> (fg.lc + k)) & 1u) << fg.hb[k];
    off[i] = o + (o & fg.gm);
  }
  auto tile_base = [&](uint64_t tile) {
    uint64_t base = tile << fg.lc;
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < fg.h) base = insert_zero(base, fg.hb[k]);
    return base + (base & fg.gm);
  };
  // software pipeline: the next tile's chunks are in flight while this tile's ops run
  chunk pf[NS][CPT];
  auto prefetch = [&](uint64_t base) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      pf[0][i] = ldc(f + base + off[i]);
      if constexpr (TWO) pf[NS - 1][i] = ldc(b + base + off[i]);
    }
  };
  const uint64_t tile0 = (uint64_t)blockIdx.x * fg.tpb;
  const uint32_t count =
      tile0 >= fg.ntiles ? 0u : (uint32_t)min<uint64_t>(fg.tpb, fg.ntiles - tile0);
  auto fill = [&]() {  // pf -> LDS, each thread its own chunks
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const uint32_t c = swz_chunk(t + (uint32_t)i * NT);
      lds[0][c] = pf[0][i];
      if constexpr (TWO) lds[NS - 1][c] = pf[NS - 1][i];
    }
  };
  uint64_t base = count ? tile_base(tile0) : 0;
  if (count) {
    prefetch(base);
    fill();
  }
  // loop rotated so the LDS refill waits (vmcnt) sit after this tile's stores in straight-line
  // code: they wait for the prefetched loads only, not for the stores issued after them
  for (uint32_t tt = 0; tt < count; ++tt) {
    __syncthreads();
    const uint64_t cur = base;
    if (tt + 1 < count) {
      base = tile_base(tile0 + tt + 1);
      prefetch(base);
    }
    uint32_t ri = 0;  // reduction op index (accumulator slot)
    for (uint32_t j = 0; j < fg.nops; ++j) {
      const fop op = ops[j];
      const uint32_t kind = op.kind & 7u;
      const bool gamma = TWO && (op.kind & FOP_GAMMA);
      const cx* M = mats + op.mat;
      if (kind == FK_Q1 || kind == FK_DENS1 || kind == FK_INJ1) {  // pairs along t1
        cx A[4], B[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) A[i] = M[i];
        if constexpr (TWO && WF) {
#pragma unroll
          for (int i = 0; i < 4; ++i) B[i] = M[4 + i];
        }
        cx acc[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        const uint32_t s1 = swz(1u << op.t1);
        const uint32_t abase = swz((uint32_t)insert_zero(t, op.t1));
#pragma unroll
        for (uint32_t it = 0; it < ta / (2 * NT); ++it) {
          const uint32_t a0 = abase ^ swz((uint32_t)insert_zero(it * NT, op.t1));
          cx fx[2] = {lf[a0], lf[a0 ^ s1]};
          if constexpr (!TWO) {
            if (kind == FK_DENS1) {
#pragma unroll
              for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                  acc[p * 2 + q] = cfma_conj(fx[p], fx[q], acc[p * 2 + q]);
              continue;
            }
          }
          if constexpr (TWO && !WF) {  // injection-only pass: b += M (2 conj f)
            const cx b0 = lb[a0], b1 = lb[a0 ^ s1];
            cx tx[2] = {{2 * fx[0].x, -2 * fx[0].y}, {2 * fx[1].x, -2 * fx[1].y}};
            umatvec<2>(A, tx);
            lb[a0] = cadd(b0, tx[0]);
            lb[a0 ^ s1] = cadd(b1, tx[1]);
            continue;
          }
          if constexpr (TWO) {
            cx bx[2] = {lb[a0], lb[a0 ^ s1]};
            if (gamma) {  // Gamma = sum b0 f0^T of the stage-entry states
#pragma unroll
              for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q) acc[p * 2 + q] = vcfma(bx[p], fx[q], acc[p * 2 + q]);
            }
            umatvec<2>(A, fx);
            umatvec<2>(B, bx);
            lb[a0] = bx[0];
            lb[a0 ^ s1] = bx[1];
          } else {
            umatvec<2>(A, fx);
          }
          lf[a0] = fx[0];
          lf[a0 ^ s1] = fx[1];
        }
        if constexpr (HASRED) {
          if (gamma || kind == FK_DENS1) {
            real v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              v[2 * i] = acc[i].x;
              v[2 * i + 1] = acc[i].y;
            }
            wave_reduce_add<8>(v, &accw[wave][ri][0]);
            ++ri;
          }
        }
      } else if (kind == FK_Q2 || kind == FK_DENS2 || kind == FK_INJ2) {  // quartets
        cx A[16], B[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) A[i] = M[i];
        if constexpr (TWO && WF) {
#pragma unroll
          for (int i = 0; i < 16; ++i) B[i] = M[16 + i];
        }
        // with several quartets per thread (NT = 128) a Gamma stage seeds acc with its first
        // product instead of zeroing it; at NT = 256 that lengthens live ranges into spills
        constexpr bool SEED = NT == 128;
        cx acc[16];
        if (!(SEED && gamma)) {
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[i] = {0, 0};
        }
        const uint32_t lo = op.t1 < op.t2 ? op.t1 : op.t2;
        const uint32_t hi = op.t1 < op.t2 ? op.t2 : op.t1;
        const uint32_t s1 = swz(1u << op.t1), s2 = swz(1u << op.t2);
        const uint32_t soff[4] = {0, s1, s2, s1 ^ s2};
        // insert_zero and swz are linear over disjoint bits: quartet it of this thread sits at
        // the thread's base XOR a uniform offset
        const uint32_t abase = swz((uint32_t)insert_zero(insert_zero(t, lo), hi));
#pragma unroll
        for (uint32_t it = 0; it < ta / (4 * NT); ++it) {
          const uint32_t a0 = abase ^ swz((uint32_t)insert_zero(insert_zero(it * NT, lo), hi));
          cx fx[4], bx[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) fx[r] = lf[a0 ^ soff[r]];
          if constexpr (!TWO) {
            if (kind == FK_DENS2) {
#pragma unroll
              for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  acc[p * 4 + q] = cfma_conj(fx[p], fx[q], acc[p * 4 + q]);
              continue;
            }
          }
          if constexpr (TWO && !WF) {  // injection-only pass: b += M (2 conj f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              bx[r] = lb[a0 ^ soff[r]];
              fx[r] = {2 * fx[r].x, -2 * fx[r].y};
            }
            umatvec<4>(A, fx);
#pragma unroll
            for (int r = 0; r < 4; ++r) lb[a0 ^ soff[r]] = cadd(bx[r], fx[r]);
            continue;
          }
          if constexpr (TWO) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bx[r] = lb[a0 ^ soff[r]];
            if (gamma) {  // Gamma = sum b0 f0^T of the stage-entry states
#pragma unroll
              for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  acc[p * 4 + q] = (SEED && it == 0) ? vcmul(bx[p], fx[q])
                                                     : vcfma(bx[p], fx[q], acc[p * 4 + q]);
            }
            umatvec<4>(A, fx);
            umatvec<4>(B, bx);
#pragma unroll
            for (int r = 0; r < 4; ++r) lb[a0 ^ soff[r]] = bx[r];
          } else {
            umatvec<4>(A, fx);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) lf[a0 ^ soff[r]] = fx[r];
        }
        if constexpr (HASRED) {
          if (gamma || kind == FK_DENS2) {
            real v[32];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              v[2 * i] = acc[i].x;
              v[2 * i + 1] = acc[i].y;
            }
            wave_reduce_add<32>(v, &accw[wave][ri][0]);
            ++ri;
          }
        }
      } else if constexpr (!(TWO && !WF)) {  // diagonal stage: A applied, B pull-back
        // quartets over (hi, lo): element r = 2 bit(hi) + bit(lo) takes diagonal entry r
        cx A[4], B[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) A[i] = M[i];
        if constexpr (TWO) {
#pragma unroll
          for (int i = 0; i < 4; ++i) B[i] = M[4 + i];
        }
        cx acc[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        const uint32_t lo = op.t1 < op.t2 ? op.t1 : op.t2;
        const uint32_t hi = op.t1 < op.t2 ? op.t2 : op.t1;
        const uint32_t s1 = swz(1u << op.t1), s2 = swz(1u << op.t2);
        const uint32_t soff[4] = {0, s1, s2, s1 ^ s2};
        const uint32_t abase = swz((uint32_t)insert_zero(insert_zero(t, lo), hi));
#pragma unroll
        for (uint32_t it = 0; it < ta / (4 * NT); ++it) {
          const uint32_t a0 = abase ^ swz((uint32_t)insert_zero(insert_zero(it * NT, lo), hi));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const cx f0 = lf[a0 ^ soff[r]];
            lf[a0 ^ soff[r]] = ucmul(A[r], f0);
            if constexpr (TWO) {
              const cx bv = lb[a0 ^ soff[r]];
              if (gamma) acc[r] = vcfma(bv, f0, acc[r]);
              lb[a0 ^ soff[r]] = ucmul(B[r], bv);
            }
          }
        }
        if constexpr (HASRED) {
          if (gamma) {
            real v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              v[2 * i] = acc[i].x;
              v[2 * i + 1] = acc[i].y;
            }
            wave_reduce_add<8>(v, &accw[wave][ri][0]);
            ++ri;
          }
        }
      }
      __syncthreads();
    }
    // each thread stores (and next refills) only its own chunks: no barrier needed here
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const uint32_t c = swz_chunk(t + (uint32_t)i * NT);
      if constexpr (WF) stc(f + cur + off[i], lds[0][c]);
      if constexpr (TWO) stc(b + cur + off[i], lds[NS - 1][c]);
    }
    if (tt + 1 < count) fill();
  }
  if constexpr (HASRED) {
    // one partial (16 complex) per block and reduction op: slot k at partials + k*slot_stride
    for (uint32_t i = t; i < fg.ngrad * FACC; i += NT) {
      const uint32_t k = i / FACC, e = i % FACC;
      real s = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) s += accw[w][k][e];
      reinterpret_cast<real*>(partials + (uint64_t)k * slot_stride + (uint64_t)blockIdx.x * RED)[e] = s;
    }
  }
}

// Read-only passes of one-qubit densities (round 6; the final densities of C2 / C5 and every
// density-only pass of a forward).  k_fused<false, TB, true, false> reduces each density of a
// tile on its own — a 64-lane reduce-scatter, an LDS accumulate and a block barrier per density
// and tile — and ran such passes at 0.30 of HBM.  Here every thread keeps its densities'
// partial sums in registers across all tiles of its block (rho11 and rho01 per density: the
// power of bit t = 1 and the cross term; rho00 = the tile power - rho11), so a tile costs two
// barriers and six FMAs per amplitude pair and density, and the block reduces once at the end.
// Same tiles (lc, h, hb, gap) and partial slots as k_fused: densities in slot order 0..nops-1,
// each partial [rho00, rho01, rho10, rho11, 0...] (rho_pq = sum f_p conj(f_q)).
constexpr int DENS1_MAX = 16;  // densities of one pass (the planner's FMAX_GRAD)
static_assert(DENS1_MAX <= FMAX_GRAD, "a density pass holds at most FMAX_GRAD densities");
template <int TB, int NT>
__global__ __launch_bounds__(NT) void k_dens1(const chunk* __restrict__ f, const fop* __restrict__ ops,
                                              fgeo fg, cx* __restrict__ partials,
                                              uint64_t slot_stride) {
  constexpr int CPT = TB / NT;  // chunks per thread and tile
  constexpr uint32_t ta = TB * VEC;  // amplitudes per tile
  static_assert(TB % NT == 0 && ta >= 2 * NT, "tile must cover the block");
  __shared__ chunk lds[TB];
  __shared__ real red[NT / 64][3 * DENS1_MAX + 1];
  const uint32_t t = threadIdx.x;
  const cx* lf = reinterpret_cast<const cx*>(&lds[0]);
  const uint32_t nops = fg.nops;  // <= DENS1_MAX (host)
  uint64_t off[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const uint32_t c = t + (uint32_t)i * NT;
    uint64_t o = c & ((1u << fg.lc) - 1u);
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < fg.h) o += (uint64_t)((c >> (fg.lc + k)) & 1u) << fg.hb[k];
    off[i] = o + (o & fg.gm);
  }
  auto tile_base = [&](uint64_t tile) {
    uint64_t base = tile << fg.lc;
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < fg.h) base = insert_zero(base, fg.hb[k]);
    return base + (base & fg.gm);
  };
  real p11[DENS1_MAX], c01r[DENS1_MAX], c01i[DENS1_MAX], ptot = 0;
#pragma unroll
  for (int j = 0; j < DENS1_MAX; ++j) p11[j] = c01r[j] = c01i[j] = 0;
  const uint64_t tile0 = (uint64_t)blockIdx.x * fg.tpb;
  const uint32_t count =
      tile0 >= fg.ntiles ? 0u : (uint32_t)min<uint64_t>(fg.tpb, fg.ntiles - tile0);
  chunk pf[CPT];
  if (count) {
    const uint64_t b0 = tile_base(tile0);
#pragma unroll
    for (int i = 0; i < CPT; ++i) pf[i] = ldc(f + b0 + off[i]);
  }
  for (uint32_t tt = 0; tt < count; ++tt) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      lds[swz_chunk(t + (uint32_t)i * NT)] = pf[i];
#pragma unroll
      for (int v = 0; v < VEC; ++v) ptot += pf[i].v[v].x * pf[i].v[v].x + pf[i].v[v].y * pf[i].v[v].y;
    }
    __syncthreads();
    if (tt + 1 < count) {  // the next tile in flight while this one is reduced
      const uint64_t nb = tile_base(tile0 + tt + 1);
#pragma unroll
      for (int i = 0; i < CPT; ++i) pf[i] = ldc(f + nb + off[i]);
    }
    // (guarded, not broken out of: the loop unrolls, so the accumulators stay in registers)
#pragma unroll
    for (int j = 0; j < DENS1_MAX; ++j) {
      if ((uint32_t)j < nops) {
        const uint32_t t1 = ops[j].t1;
        const uint32_t s1 = swz(1u << t1);
        const uint32_t abase = swz((uint32_t)insert_zero(t, t1));
#pragma unroll
        for (uint32_t it = 0; it < ta / (2 * NT); ++it) {
          const uint32_t a0 = abase ^ swz((uint32_t)insert_zero(it * NT, t1));
          const cx x0 = lf[a0], x1 = lf[a0 ^ s1];
          p11[j] = fma(x1.x, x1.x, fma(x1.y, x1.y, p11[j]));
          c01r[j] = fma(x0.x, x1.x, fma(x0.y, x1.y, c01r[j]));
          c01i[j] = fma(x0.y, x1.x, fma(-x0.x, x1.y, c01i[j]));
        }
      }
    }
    __syncthreads();
  }
  // block reduction: 64-lane sums, then the waves' sums per value
  const int lane = t & 63, wave = t >> 6;
  auto wsum = [&](real x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
  };
  {
    const real s = wsum(ptot);
    if (lane == 0) red[wave][3 * DENS1_MAX] = s;
  }
#pragma unroll
  for (int j = 0; j < DENS1_MAX; ++j) {
    if ((uint32_t)j < nops) {
      const real a = wsum(p11[j]), b = wsum(c01r[j]), c = wsum(c01i[j]);
      if (lane == 0) {
        red[wave][3 * j] = a;
        red[wave][3 * j + 1] = b;
        red[wave][3 * j + 2] = c;
      }
    }
  }
  __syncthreads();
  for (uint32_t i = t; i < nops * RED; i += NT) {
    const uint32_t k = i / RED, e = i % RED;
    real pw = 0, a = 0, b = 0, c = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      pw += red[w][3 * DENS1_MAX];
      a += red[w][3 * k];
      b += red[w][3 * k + 1];
      c += red[w][3 * k + 2];
    }
    const cx v = e == 0 ? cx{pw - a, 0} : e == 1 ? cx{b, c} : e == 2 ? cx{b, -c} : e == 3 ? cx{a, 0} : cx{0, 0};
    partials[(uint64_t)k * slot_stride + (uint64_t)blockIdx.x * RED + e] = v;
  }
}

// ---------------------------------------------------------------------------------------
// Remap pack (qdc_shard.hpp): dst block j (victim bit pattern j) = the source chunks whose
// victim bits equal j, in order.  dst[o] = src[expand(o)]: insert zeros at the victim chunk
// bits (ascending) into the low part of o, then deposit the block index bits there.  One
// chunk per thread; victims are high local bits, so every wave stays on a contiguous KiB.
// ---------------------------------------------------------------------------------------
struct packgeo {
  uint64_t nchunks;
  uint32_t lowc;   // chunk bits of one block
  uint32_t g;      // victims
  uint32_t vc[8];  // victim chunk bits, ascending
};

// UNPACK: the inverse permutation, dst[expand(o)] = src[o] (a mirrored reverse sweep undoing a
// forward remap, qdc_circuit.hpp unremap).
#ifndef QDC_SPEC_TU  // (not in the specialized kernels' translation units)
template <bool UNPACK>
__global__ __launch_bounds__(BLOCK) void k_pack(const chunk* __restrict__ src,
                                                chunk* __restrict__ dst, packgeo pg) {
  const uint64_t o = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (o >= pg.nchunks) return;
  const uint64_t j = o >> pg.lowc;
  uint64_t idx = o & ((1ull << pg.lowc) - 1ull);
  for (uint32_t k = 0; k < pg.g; ++k) idx = insert_zero(idx, pg.vc[k]);
  for (uint32_t k = 0; k < pg.g; ++k) idx |= ((j >> k) & 1ull) << pg.vc[k];
  if constexpr (UNPACK)
    stc(dst + idx, ldc(src + o));
  else
    stc(dst + o, ldc(src + idx));
}
#endif  // QDC_SPEC_TU

// The same permutations through LDS tiles (round 5).  k_pack reads (UNPACK: writes) 16 B per
// lane at victim-bit strides when a victim is a low chunk bit — and the remap planner's
// farthest-next-use victims are often qubits 1..3 — so it moved a shard at 0.7-1.3 TB/s
// (profiles/r5/r5c_shard_rehearsal.txt).  Here a block moves one tile of 2^KB chunks that is
// contiguous in the unpacked index; its image in the packed index is 2^nv runs of 2^(KB - nv)
// contiguous chunks (nv = victims below chunk bit KB <= 3), so both sides are whole-wave
// accesses of >= 1 KiB.  Tile order s ("packed order"): the tile's non-victim bits compacted
// low, its victim bits above them.
struct packtile {
  uint64_t nchunks;
  uint32_t lowc, g, vc[8];  // as packgeo
  uint32_t nv;              // victims below chunk bit PACK_KB (the first nv of vc)
};
constexpr uint32_t PACK_KB = 9;  // 512 chunks = 8 KiB of LDS per block
#ifndef QDC_SPEC_TU
template <bool UNPACK>
__global__ __launch_bounds__(256) void k_pack_tile(const chunk* __restrict__ src,
                                                   chunk* __restrict__ dst, packtile pg) {
  __shared__ chunk lds[1u << PACK_KB];
  const uint64_t base = (uint64_t)blockIdx.x << PACK_KB;  // tile base (unpacked index)
  const uint32_t lowbits = PACK_KB - pg.nv;
  auto remove_bit = [](uint64_t x, uint32_t b) {
    return (x & ((1ull << b) - 1ull)) | ((x >> (b + 1)) << b);
  };
  // tile offset t (unpacked order) <-> packed order
  auto ord = [&](uint32_t t) {
    uint32_t hi = 0;
    uint64_t x = t;
    for (int k = (int)pg.nv - 1; k >= 0; --k) {
      hi |= (uint32_t)((x >> pg.vc[k]) & 1ull) << k;
      x = remove_bit(x, pg.vc[k]);
    }
    return (uint32_t)x | (hi << lowbits);
  };
  auto inv_ord = [&](uint32_t s) {
    uint64_t x = s & ((1u << lowbits) - 1u);
    for (uint32_t k = 0; k < pg.nv; ++k) x = insert_zero(x, pg.vc[k]);
    for (uint32_t k = 0; k < pg.nv; ++k) x |= (uint64_t)((s >> (lowbits + k)) & 1u) << pg.vc[k];
    return (uint32_t)x;
  };
  // packed index of unpacked chunk index i (the inverse of k_pack's expand)
  auto packed = [&](uint64_t i) {
    uint64_t j = 0;
    for (int k = (int)pg.g - 1; k >= 0; --k) {
      j |= ((i >> pg.vc[k]) & 1ull) << k;
      i = remove_bit(i, pg.vc[k]);
    }
    return (j << pg.lowc) | i;
  };
  for (uint32_t s = threadIdx.x; s < (1u << PACK_KB); s += 256) {
    if constexpr (UNPACK)
      lds[s] = ldc(src + packed(base + inv_ord(s)));  // packed runs, in order
    else
      lds[ord(s)] = ldc(src + base + s);  // the contiguous unpacked tile
  }
  __syncthreads();
  for (uint32_t s = threadIdx.x; s < (1u << PACK_KB); s += 256) {
    if constexpr (UNPACK)
      stc(dst + base + s, lds[ord(s)]);
    else
      stc(dst + packed(base + inv_ord(s)), lds[s]);
  }
}
#endif  // QDC_SPEC_TU

// ---------------------------------------------------------------------------------------
// Elementwise state kernels (primitives.cu:176-187, 879-939).
// op 0: dst = src; op 1: dst = 2 conj(src); op 2: dst += src; op 3: dst = |0..0>; op 4: dst = 0.
// dst chunk i at i + (i & gm) (a state of an interleaved pair; src is always plain)
// ---------------------------------------------------------------------------------------
template <int OP>
__global__ __launch_bounds__(BLOCK) void k_elementwise(const cx* __restrict__ src,
                                                       cx* __restrict__ dst, uint64_t n,
                                                       uint32_t it, uint64_t gm) {
  const uint64_t nch = n / VEC;
  const chunk* s = reinterpret_cast<const chunk*>(src);
  chunk* d = reinterpret_cast<chunk*>(dst);
  const uint64_t start = (uint64_t)blockIdx.x * BLOCK * it + threadIdx.x;
  for (uint32_t step = 0; step < it; ++step) {
    const uint64_t i = start + (uint64_t)step * BLOCK;
    if (i >= nch) break;
    const uint64_t di = i + (i & gm);
    chunk a;
    if constexpr (OP == 3 || OP == 4) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) a.v[v] = (OP == 3 && i == 0 && v == 0) ? cx{1, 0} : cx{0, 0};
    } else {
      a = ldc(s + i);
    }
    if constexpr (OP == 1) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) a.v[v] = {2 * a.v[v].x, -2 * a.v[v].y};
    } else if constexpr (OP == 2) {
      const chunk o = ldc(d + di);
#pragma unroll
      for (int v = 0; v < VEC; ++v) a.v[v] = cadd(o.v[v], a.v[v]);
    }
    stc(d + di, a);
  }
  // n < VEC (a 0-qubit state in f32): scalar tail
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (uint64_t k = nch * VEC; k < n; ++k) {
      cx a = (OP == 3) ? cx{k == 0 ? (real)1 : (real)0, 0} : (OP == 4) ? cx{0, 0} : src[k];
      if constexpr (OP == 1) a = {2 * a.x, -2 * a.y};
      if constexpr (OP == 2) a = cadd(dst[k], a);
      dst[k] = a;
    }
  }
}


// Cotangent injections of a run of Diff densities whose (conjugated) cotangents are all
// diagonal (a Z-basis observable: Re tr(rho Z) and its kin).  Each injects b += (G^T on its
// qubits)(2 conj f) = 2 conj(f_i) G[k(i)][k(i)] with k(i) the density's bits of amplitude i, so
// the whole run is one elementwise pass: b_i (+)= 2 conj(f_i) D(i), D(i) = sum_g T[g][bits 4g..4g+3
// of i] (the host sums each density's diagonal into the table of the 4-bit group holding its
// qubits).  ACC = false: the run starts the backward state (no read of b, no zeroing pass).
constexpr int DI_GROUPS = 9;  // 4-bit groups of local amplitude bits 0..35
struct diag_tab {
  cx t[DI_GROUPS * 16];
};
template <bool ACC>
__global__ __launch_bounds__(BLOCK) void k_diag_inject(const chunk* __restrict__ f,
                                                       chunk* __restrict__ b, diag_tab T,
                                                       uint64_t nch, uint32_t it, uint64_t gm,
                                                       uint32_t ngroups) {
  __shared__ cx lt[DI_GROUPS * 16];
  for (uint32_t i = threadIdx.x; i < DI_GROUPS * 16; i += BLOCK) lt[i] = T.t[i];
  __syncthreads();
  const uint64_t start = (uint64_t)blockIdx.x * BLOCK * it + threadIdx.x;
  for (uint32_t step = 0; step < it; ++step) {
    const uint64_t c = start + (uint64_t)step * BLOCK;
    if (c >= nch) break;
    const uint64_t di = c + (c & gm);
    const chunk x = ldc(f + di);
    chunk o;
    if constexpr (ACC) o = ldc(b + di);
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const uint64_t a = c * VEC + v;
      cx d = lt[a & 15];
      for (uint32_t g = 1; g < ngroups; ++g) d = cadd(d, lt[g * 16 + ((a >> (4 * g)) & 15)]);
      // 2 conj(x) d
      const cx y = {2 * (x.v[v].x * d.x + x.v[v].y * d.y), 2 * (x.v[v].x * d.y - x.v[v].y * d.x)};
      o.v[v] = ACC ? cadd(o.v[v], y) : y;
    }
    stc(b + di, o);
  }
}
}  // namespace qdc
