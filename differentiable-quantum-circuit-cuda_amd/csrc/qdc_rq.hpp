// qdc_rq.hpp — register-resident fused passes (f32): the tile lives in VGPRs, LDS is only the
// exchange network between register layouts.
//
// k_fused (qdc_kernels.hpp) keeps a pass's tile in LDS and makes one LDS round trip, one
// barrier, one accumulator init and one 64-lane Gamma reduction per stage for the two quartets
// each thread owns.  At C2 n=28 that overhead is ~45 % of the reverse kernel's VALU stream, and
// the tile cannot grow: LDS (160 KiB/CU) is what bounds occupancy.  Here each thread holds
// R = 16 amplitudes of every state in registers (the VGPR file is 512 KiB/CU): 4 "register
// qubits" (slots 0..3) and log2(NT) "thread qubits".  A stage whose qubits sit in register
// slots runs on registers only, over 4 quartets per thread (8 one-qubit pairs): no LDS, no
// barrier, twice the quartets per Gamma reduction.  When the next stage needs other qubits in
// registers, a RELAYOUT op writes the state to LDS in the current layout and reads it back in
// the new one (one state at a time through one buffer, so a block needs 2^T * 8 B of LDS).
// The host (qdc_fusion.hpp, rq_plan) chooses the layouts: slots form two pairs {0,1}, {2,3};
// a two-qubit stage occupies one pair (either orientation), a one-qubit stage any slot, and
// the slot pair (or slot) to replace is the one whose qubits are needed again last.
//
// Layout L: tile bits of slots 0..3 plus the remaining tile bits as thread bits (ascending).
// Amplitude (thread t, register j) sits at tile index dep(t -> thread bits) | dep(j -> slots).
// LDS index = swz(...) = swz(dep(t)) ^ swz(dep(j)): a per-thread part tp (from the layout's
// swizzled thread-bit vectors tv[]) XOR a uniform part rp[j].  L0 (load/store layout): slot 0 =
// tile bit 0 (the two amplitudes of a 16-B chunk), slots 1..3 = the top three tile bits, thread
// bits = tile bits 1..T-4 — so register pair (2i, 2i+1) is chunk t + i*NT, as in k_fused, and
// loads/stores go straight between HBM and registers.  Every program ends in L0.
#pragma once

#include <type_traits>

#include "qdc_kernels.hpp"

namespace qdc {

#ifndef QDC_RQ_GSPLIT
#define QDC_RQ_GSPLIT 0
#endif
// register stages apply their matrices to two quartets (four pairs) at once, the dependency
// chains interleaved (umatvec_n); 0: one quartet (pair) at a time (rounds 1-4).  Same box,
// bit-identical: 4660-4668 vs 4651 gates/s (profiles/r5/r5d_pk_forms_ab.txt)
#ifndef QDC_MATVEC_N
#define QDC_MATVEC_N 1
#endif

constexpr int RQ_R = 16;  // amplitudes per thread per state
constexpr uint32_t FK_RELAYOUT = 7;
constexpr int RQ_NT_ONE = 256;  // threads per one-state tile: 2^12 amplitudes = TILE_CHUNKS_1
constexpr int RQ_NT_TWO = 128;  // threads per two-state tile: 2^11 amplitudes = TILE_CHUNKS_2

// a register layout in the program's matrix area (160 B: 20 cx in f32, 10 in f64); 4-slot
// layouts use rp[0..15], 5-slot ones (k_rw two-state f32) rp[0..31]
struct rq_layout {
  uint32_t rp[2 * RQ_R];  // swz(dep(j -> slots)), in cx units
  uint32_t tv[8];         // swz(1 << thread bit k), in cx units (k < log2 NT)
};
static_assert(sizeof(rq_layout) == 160 && sizeof(rq_layout) % sizeof(cx) == 0,
              "rq_layout is whole complex values of the program");

// HBM addressing of a tile's registers (after the load layout's descriptor in the program).
// Register pair (2i, 2i+1) of thread t is one 16-B chunk (slot 0 = tile bit 0); its chunk
// offset from the tile base is thr(t) + offi[i], thr(t) = sum of gv[k] over the set bits k of
// t (thread bit k's chunk offset) and offi[i] = the offset of register chunk bits i (slots 1..3).
// The load layout (the pass's first) and the store layout (its last) may differ.
struct rqio {
  uint64_t gv_ld[8], offi_ld[RQ_R], gv_st[8], offi_st[RQ_R];  // offi: RQ_R / VEC chunks used
};
static_assert(sizeof(rqio) % sizeof(cx) == 0, "rqio is whole complex values of the program");

// Everything below builds in both precisions; k_rq and the prefetch loads are f32 only (never
// instantiated by the f64 runtime), k_rw runs both.

// fop.t1 of a register stage = slot case (rq_stage); register index bit s = slot s.
template <int S1, int S2>
__device__ __forceinline__ constexpr int rq_el(int base, int r) {
  return base | ((r & 1) << S1) | ((r >> 1) << S2);
}
template <int S1, int S2>
__device__ __forceinline__ constexpr int rq_base(int k) {  // k-th index with bits S1, S2 zero
  int b = 0, bit = 0;
  for (int s = 0; s < 8; ++s) {  // the register index bits other than S1, S2, ascending
    if (s == S1 || s == S2) continue;
    if ((k >> bit) & 1) b |= 1 << s;
    ++bit;
  }
  return b;
}

// two-qubit stage on registers: f <- A f [, Gamma += b0 f0^T, b <- B b]
template <int S1, int S2, bool TWO, int R>
__device__ __forceinline__ void rq_q2(cx (&f)[R], cx (&b)[R], const cx* __restrict__ M,
                                      bool gamma, real* acc_out) {
  cx A[16], B[16];
  if (TWO && gamma) {
    // QDC_RQ_GSPLIT: Gamma in two halves of rows (p = 0, 1 then 2, 3), each reduced on its own:
    // 16 accumulator VGPRs live instead of 32 at the same reduce-scatter cost (two 16-value
    // reductions ~ one of 32), for register pressure at the 256-VGPR limit
    constexpr int NH = (QDC_RQ_GSPLIT && R >= 32) ? 2 : 1;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      constexpr int PR = 4 / NH;  // rows per half
      cx acc[4 * PR];
#pragma unroll
      for (int k = 0; k < R / 4; ++k) {
        const int base = rq_base<S1, S2>(k);
#pragma unroll
        for (int pp = 0; pp < PR; ++pp)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int p = h * PR + pp;
            const cx bp = b[rq_el<S1, S2>(base, p)], fq = f[rq_el<S1, S2>(base, q)];
            acc[pp * 4 + q] = k == 0 ? vcmul(bp, fq) : vcfma(bp, fq, acc[pp * 4 + q]);
          }
      }
      real v[8 * PR];
#pragma unroll
      for (int i = 0; i < 4 * PR; ++i) {
        v[2 * i] = acc[i].x;
        v[2 * i + 1] = acc[i].y;
      }
      wave_reduce_add<8 * PR>(v, acc_out + h * 8 * PR);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) A[i] = M[i];
  // f with A, then b with B: one matrix (32 SGPRs) live at a time; two quartets at once (8
  // interleaved dependency chains: no hazard padding between the packed FMAs, umatvec_n)
  constexpr int NQ = (QDC_MATVEC_N && R / 4 >= 2) ? 2 : 1;
#pragma unroll
  for (int k = 0; k < R / 4; k += NQ) {
    cx x[NQ][4];
#pragma unroll
    for (int n = 0; n < NQ; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) x[n][r] = f[rq_el<S1, S2>(rq_base<S1, S2>(k + n), r)];
    umatvec_n<4, NQ>(A, x);
#pragma unroll
    for (int n = 0; n < NQ; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) f[rq_el<S1, S2>(rq_base<S1, S2>(k + n), r)] = x[n][r];
  }
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < 16; ++i) B[i] = M[16 + i];
#pragma unroll
    for (int k = 0; k < R / 4; k += NQ) {
      cx x[NQ][4];
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[n][r] = b[rq_el<S1, S2>(rq_base<S1, S2>(k + n), r)];
      umatvec_n<4, NQ>(B, x);
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) b[rq_el<S1, S2>(rq_base<S1, S2>(k + n), r)] = x[n][r];
    }
  }
}

// diagonal two-qubit stage: element r = 2 bit(t2) + bit(t1) of each quartet takes entry r
template <int S1, int S2, bool TWO, int R>
__device__ __forceinline__ void rq_diag(cx (&f)[R], cx (&b)[R], const cx* __restrict__ M,
                                        bool gamma, real* acc_out) {
  cx A[4], B[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) A[i] = M[i];
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < 4; ++i) B[i] = M[4 + i];
  }
  if (TWO && gamma) {
    cx acc[4];
#pragma unroll
    for (int k = 0; k < R / 4; ++k) {
      const int base = rq_base<S1, S2>(k);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = rq_el<S1, S2>(base, r);
        acc[r] = k == 0 ? vcmul(b[e], f[e]) : vcfma(b[e], f[e], acc[r]);
      }
    }
    real v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = acc[i].x;
      v[2 * i + 1] = acc[i].y;
    }
    wave_reduce_add<8>(v, acc_out);
  }
#pragma unroll
  for (int k = 0; k < R / 4; ++k) {
    const int base = rq_base<S1, S2>(k);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = rq_el<S1, S2>(base, r);
      f[e] = ucmul(A[r], f[e]);
      if constexpr (TWO) b[e] = ucmul(B[r], b[e]);
    }
  }
}

// one-qubit stage on slot S: pairs (j, j | 1 << S)
template <int S, bool TWO, int R>
__device__ __forceinline__ void rq_q1(cx (&f)[R], cx (&b)[R], const cx* __restrict__ M,
                                      bool gamma, real* acc_out) {
  cx A[4], B[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) A[i] = M[i];
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < 4; ++i) B[i] = M[4 + i];
  }
  constexpr int LOWM = (1 << S) - 1;
  if (TWO && gamma) {
    cx acc[4];
#pragma unroll
    for (int k = 0; k < R / 2; ++k) {
      const int j0 = ((k & ~LOWM) << 1) | (k & LOWM), j1 = j0 | (1 << S);
      const cx bx[2] = {b[j0], b[j1]}, fx[2] = {f[j0], f[j1]};
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          acc[p * 2 + q] = k == 0 ? vcmul(bx[p], fx[q]) : vcfma(bx[p], fx[q], acc[p * 2 + q]);
    }
    real v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = acc[i].x;
      v[2 * i + 1] = acc[i].y;
    }
    wave_reduce_add<8>(v, acc_out);
  }
  // four pairs at once (8 interleaved dependency chains, umatvec_n)
  constexpr int NP = (QDC_MATVEC_N && R / 2 >= 4) ? 4 : 1;
#pragma unroll
  for (int k = 0; k < R / 2; k += NP) {
    cx x[NP][2];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      const int j0 = (((k + n) & ~LOWM) << 1) | ((k + n) & LOWM), j1 = j0 | (1 << S);
      x[n][0] = f[j0];
      x[n][1] = f[j1];
    }
    umatvec_n<2, NP>(A, x);
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      const int j0 = (((k + n) & ~LOWM) << 1) | ((k + n) & LOWM), j1 = j0 | (1 << S);
      f[j0] = x[n][0];
      f[j1] = x[n][1];
    }
    if constexpr (TWO) {
#pragma unroll
      for (int n = 0; n < NP; ++n) {
        const int j0 = (((k + n) & ~LOWM) << 1) | ((k + n) & LOWM), j1 = j0 | (1 << S);
        x[n][0] = b[j0];
        x[n][1] = b[j1];
      }
      umatvec_n<2, NP>(B, x);
#pragma unroll
      for (int n = 0; n < NP; ++n) {
        const int j0 = (((k + n) & ~LOWM) << 1) | ((k + n) & LOWM), j1 = j0 | (1 << S);
        b[j0] = x[n][0];
        b[j1] = x[n][1];
      }
    }
  }
}

// one register stage: slot case (host: rq_plan) two-qubit / diagonal S1 * 8 + S2 (t1 in slot
// S1, t2 in slot S2, always S1 < S2: build_program exchanges t1 and t2 otherwise); one-qubit:
// the slot of t1
template <bool TWO, int R>
__device__ __forceinline__ void rq_stage(uint32_t sel, cx (&xf)[R], cx (&xb)[R],
                                         const cx* __restrict__ M, bool gamma, real* acc) {
  // slot 4 exists only with 32 registers (five-slot layouts)
#define QDC_RQ_Q2(S1, S2)                                                             \
  case FK_Q2 * 64 + (S1) * 8 + (S2):                                                  \
    if constexpr ((S2) < 4 || R >= 32) rq_q2<S1, S2, TWO, R>(xf, xb, M, gamma, acc);   \
    break;                                                                            \
  case FK_DIAG * 64 + (S1) * 8 + (S2):                                                \
    if constexpr ((S2) < 4 || R >= 32) rq_diag<S1, S2, TWO, R>(xf, xb, M, gamma, acc); \
    break;
  switch (sel) {
    QDC_RQ_Q2(0, 1) QDC_RQ_Q2(0, 2) QDC_RQ_Q2(0, 3) QDC_RQ_Q2(1, 2) QDC_RQ_Q2(1, 3)
    QDC_RQ_Q2(2, 3) QDC_RQ_Q2(0, 4) QDC_RQ_Q2(1, 4) QDC_RQ_Q2(2, 4) QDC_RQ_Q2(3, 4)
    case FK_Q1 * 64 + 0: rq_q1<0, TWO, R>(xf, xb, M, gamma, acc); break;
    case FK_Q1 * 64 + 1: rq_q1<1, TWO, R>(xf, xb, M, gamma, acc); break;
    case FK_Q1 * 64 + 2: rq_q1<2, TWO, R>(xf, xb, M, gamma, acc); break;
    case FK_Q1 * 64 + 4:
      if constexpr (R >= 32) rq_q1<4, TWO, R>(xf, xb, M, gamma, acc);
      break;
    default: rq_q1<3, TWO, R>(xf, xb, M, gamma, acc); break;
  }
#undef QDC_RQ_Q2
}

// per-thread part of a layout's LDS index
template <int LOGNT>
__device__ __forceinline__ uint32_t rq_tp(const rq_layout* L, uint32_t t) {
  uint32_t tp = 0;
#pragma unroll
  for (int k = 0; k < LOGNT; ++k) tp ^= ((t >> k) & 1u) ? L->tv[k] : 0u;
  return tp;
}

// move one state from layout (tp, Lc) to (tpn, Ln) through the LDS buffer
__device__ __forceinline__ void rq_exchange(cx (&x)[RQ_R], cx* buf, uint32_t tp,
                                            const rq_layout* Lc, uint32_t tpn,
                                            const rq_layout* Ln) {
#if !(QDC_RQ_ABL & 16)
  __syncthreads();  // every thread is done reading the buffer's previous contents
#endif
  // byte addressing with the uniform part scaled on the scalar unit: one v_xor per access
  // (opaque per-thread parts: LLVM would refactor (a*8)^(b*8) back into (a^b)*8)
  char* const bufb = reinterpret_cast<char*>(buf);
  uint32_t tpb = tp * (uint32_t)sizeof(cx), tpnb = tpn * (uint32_t)sizeof(cx);
  asm volatile("" : "+v"(tpb), "+v"(tpnb));
#pragma unroll
  for (int j = 0; j < RQ_R; ++j)
    *reinterpret_cast<cx*>(__builtin_assume_aligned(bufb + (tpb ^ (Lc->rp[j] * (uint32_t)sizeof(cx))), 8)) = x[j];
#if !(QDC_RQ_ABL & 16)
  __syncthreads();
#endif
#pragma unroll
  for (int j = 0; j < RQ_R; ++j)
    x[j] = *reinterpret_cast<const cx*>(
        __builtin_assume_aligned(bufb + (tpnb ^ (Ln->rp[j] * (uint32_t)sizeof(cx))), 8));
}

// Prefetch loads the compiler's waitcnt pass does not see.  With ordinary loads it drains the
// whole prefetch (s_waitcnt vmcnt(0)) at the first stage of the pass loop: a loop that reads
// registers loaded outside it gets its vector-memory counter flushed, so the next tile's
// loads never overlapped this tile's stages.  These loads are waited for explicitly (counted:
// the wave's younger vector-memory ops are known at every wait).  Their destinations are fixed
// physical VGPRs, the same in the load and in the wait (a tied in/out operand of the wait
// asm), so the register allocator never has a reason to copy an in-flight register: a copy
// before the wait would read stale data.  tools/check_rq_isa.py checks the ISA for any read
// of them between a load and its wait.
// Pinned registers: one-state passes v[96:127] (8 chunks), two-state v[192:255] (16 chunks).
constexpr int RQ_PIN_ONE = 96, RQ_PIN_TWO = 192;
template <int REG>
__device__ __forceinline__ vec16 rq_ld(const chunk* p) {
  vec16 v;
  switch (REG) {
    case 96: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[96:99]}"(v) : "v"(p) : "memory"); break;
    case 100: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[100:103]}"(v) : "v"(p) : "memory"); break;
    case 104: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[104:107]}"(v) : "v"(p) : "memory"); break;
    case 108: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[108:111]}"(v) : "v"(p) : "memory"); break;
    case 112: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[112:115]}"(v) : "v"(p) : "memory"); break;
    case 116: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[116:119]}"(v) : "v"(p) : "memory"); break;
    case 120: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[120:123]}"(v) : "v"(p) : "memory"); break;
    case 124: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[124:127]}"(v) : "v"(p) : "memory"); break;
    case 192: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[192:195]}"(v) : "v"(p) : "memory"); break;
    case 196: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[196:199]}"(v) : "v"(p) : "memory"); break;
    case 200: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[200:203]}"(v) : "v"(p) : "memory"); break;
    case 204: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[204:207]}"(v) : "v"(p) : "memory"); break;
    case 208: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[208:211]}"(v) : "v"(p) : "memory"); break;
    case 212: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[212:215]}"(v) : "v"(p) : "memory"); break;
    case 216: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[216:219]}"(v) : "v"(p) : "memory"); break;
    case 220: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[220:223]}"(v) : "v"(p) : "memory"); break;
    case 224: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[224:227]}"(v) : "v"(p) : "memory"); break;
    case 228: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[228:231]}"(v) : "v"(p) : "memory"); break;
    case 232: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[232:235]}"(v) : "v"(p) : "memory"); break;
    case 236: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[236:239]}"(v) : "v"(p) : "memory"); break;
    case 240: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[240:243]}"(v) : "v"(p) : "memory"); break;
    case 244: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[244:247]}"(v) : "v"(p) : "memory"); break;
    case 248: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[248:251]}"(v) : "v"(p) : "memory"); break;
    case 252: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={v[252:255]}"(v) : "v"(p) : "memory"); break;
  }
  return v;
}
// vmcnt(0) on a wave's first tile (nothing issued after its loads), else vmcnt(N)
#define QDC_RQ_WAIT_ASM                                     \
  "s_cmp_eq_u32 %[first], 0\n\t"                           \
  "s_cbranch_scc1 1f\n\t"                                  \
  "s_waitcnt vmcnt(0)\n\t"                                 \
  "s_branch 2f\n"                                           \
  "1:\n\t"                                                 \
  "s_waitcnt vmcnt(%[cnt])\n"                               \
  "2:"
template <int N>
__device__ __forceinline__ void rq_vmwait_one(uint32_t first, vec16 (&v)[8]) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  const uint32_t fs = __builtin_amdgcn_readfirstlane(first);
  asm volatile(QDC_RQ_WAIT_ASM
               : "+{v[96:99]}"(v[0]), "+{v[100:103]}"(v[1]), "+{v[104:107]}"(v[2]), "+{v[108:111]}"(v[3]), "+{v[112:115]}"(v[4]), "+{v[116:119]}"(v[5]), "+{v[120:123]}"(v[6]), "+{v[124:127]}"(v[7])
               : [first] "s"(fs), [cnt] "n"(N)
               : "memory", "scc");
}
template <int N>
__device__ __forceinline__ void rq_vmwait_two(uint32_t first, vec16 (&v)[8], vec16 (&w)[8]) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  const uint32_t fs = __builtin_amdgcn_readfirstlane(first);
  asm volatile(QDC_RQ_WAIT_ASM
               : "+{v[192:195]}"(v[0]), "+{v[196:199]}"(v[1]), "+{v[200:203]}"(v[2]), "+{v[204:207]}"(v[3]), "+{v[208:211]}"(v[4]), "+{v[212:215]}"(v[5]), "+{v[216:219]}"(v[6]), "+{v[220:223]}"(v[7]),
                 "+{v[224:227]}"(w[0]), "+{v[228:231]}"(w[1]), "+{v[232:235]}"(w[2]), "+{v[236:239]}"(w[3]), "+{v[240:243]}"(w[4]), "+{v[244:247]}"(w[5]), "+{v[248:251]}"(w[6]), "+{v[252:255]}"(w[7])
               : [first] "s"(fs), [cnt] "n"(N)
               : "memory", "scc");
}


// k_rw prefetch: the next tile's 32 chunks in AGPRs a[0:127] (one wave per SIMD: 256 VGPRs +
// 256 AGPRs), loaded and waited for as in rq_ld / rq_vmwait_two (hidden from the waitcnt pass,
// pinned registers, a tied wait).  The wait covers all 32 chunks; the second statement only
// re-defines a[64:127] after it (asm volatile statements keep their order).
template <int REG>
__device__ __forceinline__ vec16 rw_lda(const chunk* p) {
  vec16 v;
  switch (REG) {
    case 0: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[0:3]}"(v) : "v"(p) : "memory"); break;
    case 4: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[4:7]}"(v) : "v"(p) : "memory"); break;
    case 8: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[8:11]}"(v) : "v"(p) : "memory"); break;
    case 12: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[12:15]}"(v) : "v"(p) : "memory"); break;
    case 16: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[16:19]}"(v) : "v"(p) : "memory"); break;
    case 20: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[20:23]}"(v) : "v"(p) : "memory"); break;
    case 24: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[24:27]}"(v) : "v"(p) : "memory"); break;
    case 28: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[28:31]}"(v) : "v"(p) : "memory"); break;
    case 32: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[32:35]}"(v) : "v"(p) : "memory"); break;
    case 36: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[36:39]}"(v) : "v"(p) : "memory"); break;
    case 40: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[40:43]}"(v) : "v"(p) : "memory"); break;
    case 44: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[44:47]}"(v) : "v"(p) : "memory"); break;
    case 48: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[48:51]}"(v) : "v"(p) : "memory"); break;
    case 52: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[52:55]}"(v) : "v"(p) : "memory"); break;
    case 56: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[56:59]}"(v) : "v"(p) : "memory"); break;
    case 60: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[60:63]}"(v) : "v"(p) : "memory"); break;
    case 64: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[64:67]}"(v) : "v"(p) : "memory"); break;
    case 68: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[68:71]}"(v) : "v"(p) : "memory"); break;
    case 72: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[72:75]}"(v) : "v"(p) : "memory"); break;
    case 76: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[76:79]}"(v) : "v"(p) : "memory"); break;
    case 80: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[80:83]}"(v) : "v"(p) : "memory"); break;
    case 84: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[84:87]}"(v) : "v"(p) : "memory"); break;
    case 88: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[88:91]}"(v) : "v"(p) : "memory"); break;
    case 92: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[92:95]}"(v) : "v"(p) : "memory"); break;
    case 96: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[96:99]}"(v) : "v"(p) : "memory"); break;
    case 100: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[100:103]}"(v) : "v"(p) : "memory"); break;
    case 104: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[104:107]}"(v) : "v"(p) : "memory"); break;
    case 108: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[108:111]}"(v) : "v"(p) : "memory"); break;
    case 112: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[112:115]}"(v) : "v"(p) : "memory"); break;
    case 116: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[116:119]}"(v) : "v"(p) : "memory"); break;
    case 120: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[120:123]}"(v) : "v"(p) : "memory"); break;
    case 124: asm volatile("global_load_dwordx4 %0, %1, off nt" : "={a[124:127]}"(v) : "v"(p) : "memory"); break;
  }
  return v;
}
template <int N>
__device__ __forceinline__ void rw_vmwait(uint32_t first, vec16 (&v)[32]) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  const uint32_t fs = __builtin_amdgcn_readfirstlane(first);
  asm volatile(QDC_RQ_WAIT_ASM
               : "+{a[0:3]}"(v[0]), "+{a[4:7]}"(v[1]), "+{a[8:11]}"(v[2]), "+{a[12:15]}"(v[3]), "+{a[16:19]}"(v[4]), "+{a[20:23]}"(v[5]), "+{a[24:27]}"(v[6]), "+{a[28:31]}"(v[7]), "+{a[32:35]}"(v[8]), "+{a[36:39]}"(v[9]), "+{a[40:43]}"(v[10]), "+{a[44:47]}"(v[11]), "+{a[48:51]}"(v[12]), "+{a[52:55]}"(v[13]), "+{a[56:59]}"(v[14]), "+{a[60:63]}"(v[15])
               : [first] "s"(fs), [cnt] "n"(N)
               : "memory", "scc");
  asm volatile(""
               : "+{a[64:67]}"(v[16]), "+{a[68:71]}"(v[17]), "+{a[72:75]}"(v[18]), "+{a[76:79]}"(v[19]), "+{a[80:83]}"(v[20]), "+{a[84:87]}"(v[21]), "+{a[88:91]}"(v[22]), "+{a[92:95]}"(v[23]), "+{a[96:99]}"(v[24]), "+{a[100:103]}"(v[25]), "+{a[104:107]}"(v[26]), "+{a[108:111]}"(v[27]), "+{a[112:115]}"(v[28]), "+{a[116:119]}"(v[29]), "+{a[120:123]}"(v[30]), "+{a[124:127]}"(v[31])
               :
               : "memory");
}

// TWO: fwd and bwd (reverse sweep, Gamma stages reduce into partials); else fwd only.
// fg.nops ops at `ops`; at mats + l0 the load layout's descriptor, then rqio.
#ifndef QDC_RQ_PF_WAVES
#define QDC_RQ_PF_WAVES 2  // waves/SIMD of the prefetching variant (state + next tile in VGPRs)
#endif
// PF: software pipeline — the next tile's chunks are loaded into registers while this tile's
// stages run (2x the state registers, so fewer waves).
// PROG (not void): the pass program as a functor of straight-line stage calls (qdc_spec.hpp,
// one-state specialized passes) in place of the interpreted op loop; everything else the same.
struct SpecEnv {
  const cx* mats;
  const fop* ops;
  real (*accw)[FACC];  // two-state: the Gamma stage accumulators
  uint32_t t;          // the block's thread
  char* bufb;          // the relayout buffer
};
template <bool TWO, int NT, bool PF, class PROG = void>
__device__ __forceinline__ void rq_pass(chunk* __restrict__ f, chunk* __restrict__ b,
                                        const fop* __restrict__ ops, const cx* __restrict__ mats,
                                        fgeo fg, uint32_t l0, cx* __restrict__ partials,
                                        uint64_t slot_stride) {
  constexpr int LOGNT = NT == 64 ? 6 : NT == 128 ? 7 : NT == 256 ? 8 : 9;
  constexpr int CPT = RQ_R / VEC;  // chunks of each state per thread (8)
  constexpr int TA = NT * RQ_R;    // amplitudes per tile and state
  __shared__ cx buf[TA];
  __shared__ real accw[TWO ? NT / 64 : 1][TWO ? FMAX_GRAD_RQ : 1][FACC];
  const uint32_t t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane((int)(t >> 6));
  if constexpr (TWO) {
    for (uint32_t i = t; i < (NT / 64) * FMAX_GRAD_RQ * FACC; i += NT) (&accw[0][0][0])[i] = 0;
    // a wave's accumulators are zeroed partly by other waves; a Gamma stage can come before
    // the pass's first relayout barrier
    __syncthreads();
  }
  const rq_layout* L0 = reinterpret_cast<const rq_layout*>(mats + l0);
  const rqio* io = reinterpret_cast<const rqio*>(mats + l0 + sizeof(rq_layout) / sizeof(cx));
  uint64_t thr_ld = 0, thr_st = 0;  // this thread's chunk offsets in the load / store layout
#pragma unroll
  for (int k = 0; k < LOGNT; ++k) {
    if ((t >> k) & 1u) {
      thr_ld += io->gv_ld[k];
      thr_st += io->gv_st[k];
    }
  }
  // block-contiguous tiles (tile0 + s) or grid-strided (tile0 + s * grid: concurrently running
  // tiles are neighbours in memory)
  const bool gstride = fg.order == 1;  // 2: block-contiguous in XCD-aware block order
  const uint64_t tile0 = gstride ? (uint64_t)blockIdx.x
                                 : (uint64_t)xcd_block(blockIdx.x, gridDim.x, fg.order == 2) * fg.tpb;
  const uint64_t tstep = gstride ? (uint64_t)gridDim.x : 1u;
  // static share (all tiles, or tpb of the first nstat with a dynamic tail: one-state PF only)
  const uint64_t nst = (QDC_DYN_TAIL && PF && !TWO && fg_arg()->ndyn) ? fg_arg()->nstat : fg.ntiles;
  const uint32_t count =
      tile0 >= nst ? 0u
      : gstride    ? (uint32_t)((nst - 1 - tile0) / tstep + 1)
                   : (uint32_t)min<uint64_t>(fg.tpb, nst - tile0);
  // (geometry read through the kernarg pointer at each use: held in SGPRs across the pass it was
  // spilled to VGPR lanes and this ran on the VALU)
  auto tile_base = [&](uint64_t tile) {
    const fg_kptr a = fg_arg();
    uint64_t base = tile << a->lc;
    const uint32_t h = a->h;
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < h) base = insert_zero(base, a->hb[k]);
    return base + (base & a->gm);
  };
  // re-read per use, so the compiler does not hold the offsets in SGPRs across the pass
  auto rqio_now = [&]() {
    uint32_t ro = l0;
    asm volatile("" : "+s"(ro));
    return reinterpret_cast<const rqio*>(mats + ro + sizeof(rq_layout) / sizeof(cx));
  };
  auto load = [&](cx (&xf)[RQ_R], cx (&xb)[RQ_R], uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    const chunk* pf = f + (base + thr_ld);
    const chunk* pb = b + (base + thr_ld);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const chunk cf = ldc(pf + rg->offi_ld[i]);
      xf[2 * i] = cf.v[0];
      xf[2 * i + 1] = cf.v[1];
      if constexpr (TWO) {
        const chunk cb = ldc(pb + rg->offi_ld[i]);
        xb[2 * i] = cb.v[0];
        xb[2 * i + 1] = cb.v[1];
      }
    }
  };
  // the program ends in the store layout.  The opaque redefinition keeps the compiler from
  // holding the loads' 16 addresses across the pass.
  auto store = [&](cx (&xf)[RQ_R], cx (&xb)[RQ_R], uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    chunk* pf = f + (base + thr_st);
    chunk* pb = b + (base + thr_st);
    asm volatile("" : "+v"(pf), "+v"(pb));
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      chunk c;
      c.v[0] = xf[2 * i];
      c.v[1] = xf[2 * i + 1];
      stc(pf + rg->offi_st[i], c);
      if constexpr (TWO) {
        c.v[0] = xb[2 * i];
        c.v[1] = xb[2 * i + 1];
        stc(pb + rg->offi_st[i], c);
      }
    }
  };
  auto run = [&](cx (&xf)[RQ_R], cx (&xb)[RQ_R]) __attribute__((always_inline)) {
    if constexpr (!std::is_same<PROG, void>::value) {
      static_assert(!TWO, "specialized passes of k_rq: one-state");
      PROG{}(xf, SpecEnv{mats, ops, nullptr, t, reinterpret_cast<char*>(buf)});
      return;
    }
    // loop state kept small (register pressure): the current layout as a uniform offset into
    // the program; the per-thread LDS parts are recomputed at each relayout
    uint32_t lcur = l0;
    uint32_t tpc = TWO ? 0u : rq_tp<LOGNT>(reinterpret_cast<const rq_layout*>(mats + l0), t);
    uint32_t ri = 0;
    for (uint32_t j = 0; j < fg.nops; ++j) {
      const fop op = ops[j];
      const uint32_t kind = op.kind & 7u;
      const bool gamma = TWO && (op.kind & FOP_GAMMA) && !(QDC_RQ_ABL & 4);
      const cx* M = mats + op.mat;
      // ri < FMAX_GRAD_RQ: build_program rejects a pass with more Gamma stages
      real* acc = TWO ? &accw[wave][ri][0] : nullptr;
      if ((QDC_RQ_ABL & 2) && kind == FK_RELAYOUT) {
        lcur = op.mat;
        continue;
      }
      if ((QDC_RQ_ABL & 1) && kind != FK_RELAYOUT) {
        if (TWO && (op.kind & FOP_GAMMA)) ++ri;
        continue;
      }
      if (kind == FK_RELAYOUT) {
        const rq_layout* Lc = reinterpret_cast<const rq_layout*>(mats + lcur);
        const rq_layout* Ln = reinterpret_cast<const rq_layout*>(M);
        // two-state: recomputed (register pressure); one-state: carried
        const uint32_t tp = TWO ? rq_tp<LOGNT>(Lc, t) : tpc, tpn = rq_tp<LOGNT>(Ln, t);
        rq_exchange(xf, buf, tp, Lc, tpn, Ln);
        if constexpr (TWO) rq_exchange(xb, buf, tp, Lc, tpn, Ln);
        tpc = tpn;
        lcur = op.mat;
        continue;
      }
      rq_stage<TWO>(kind * 64u + op.t1, xf, xb, M, gamma, acc);
      if (gamma) ++ri;
    }
  };
  if constexpr (!PF) {
    cx xf[RQ_R], xb[RQ_R];
    for (uint32_t tt = 0; tt < count; ++tt) {
      const uint64_t base = tile_base(tile0 + tt * tstep);
      load(xf, xb, base);
      run(xf, xb);
      store(xf, xb, base);
    }
  } else {
    // the next tile's chunks (pf_f, pf_b) are in flight while this tile (xf, xb) runs
    constexpr int NLD = TWO ? 2 * CPT : CPT;  // vector-memory ops per tile: loads = stores
    vec16 pf_f[CPT], pf_b[CPT];
    cx xf[RQ_R], xb[RQ_R];
    auto issue = [&](uint64_t base) __attribute__((always_inline)) {
      const rqio* rg = rqio_now();
      const chunk* pf = f + (base + thr_ld);
      const chunk* pb = b + (base + thr_ld);
      constexpr int BASE = TWO ? RQ_PIN_TWO : RQ_PIN_ONE;
#define QDC_RQ_ISSUE(i)                                                                   \
  pf_f[i] = rq_ld<BASE + 4 * (i)>(pf + rg->offi_ld[i]);                                   \
  if constexpr (TWO) pf_b[i] = rq_ld<RQ_PIN_TWO + 32 + 4 * (i)>(pb + rg->offi_ld[i]);
      static_assert(CPT == 8, "eight chunks per state and thread");
      QDC_RQ_ISSUE(0) QDC_RQ_ISSUE(1) QDC_RQ_ISSUE(2) QDC_RQ_ISSUE(3)
      QDC_RQ_ISSUE(4) QDC_RQ_ISSUE(5) QDC_RQ_ISSUE(6) QDC_RQ_ISSUE(7)
#undef QDC_RQ_ISSUE
    };
    auto take = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const chunk c = __builtin_bit_cast(chunk, pf_f[i]);
        xf[2 * i] = c.v[0];
        xf[2 * i + 1] = c.v[1];
        if constexpr (TWO) {
          const chunk d = __builtin_bit_cast(chunk, pf_b[i]);
          xb[2 * i] = d.v[0];
          xb[2 * i + 1] = d.v[1];
        }
      }
    };
    // Dynamic tail (one-state passes, fgeo::ndyn): after its count static tiles the block takes
    // tiles from its pool's counter.  Thread 0 grabs step s+1's tile during step s — the atomic
    // is older than that step's stores, so the compiler's own wait for its result is vmcnt(#
    // stores) and never drains the pipeline — and hands it to the block through LDS.
    __shared__ uint64_t grab_sh;
    unsigned long long grabbed = 0;  // thread 0: the counter value of the grab in flight
    const bool dyn = QDC_DYN_TAIL && !TWO && fg_arg()->ndyn != 0;
    const uint64_t per = dyn ? fg_arg()->ndyn >> 3 : 0;
    const uint64_t pool0 = fg_arg()->nstat + (uint64_t)(blockIdx.x & 7u) * per;
    auto grab_issue = [&]() __attribute__((always_inline)) {
      if (t == 0) grabbed = atomicAdd(fg_arg()->dctr + FG_DCTR_STRIDE * (blockIdx.x & 7u), 1ull);
    };
    auto grab_take = [&]() __attribute__((always_inline)) {  // block-uniform: k-th pool tile
      __syncthreads();  // every thread read the previous grab
      if (t == 0) grab_sh = (uint64_t)grabbed - fg_arg()->dbase;
      __syncthreads();
      const uint64_t k = grab_sh;
      return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(k >> 32)) << 32) |
             __builtin_amdgcn_readfirstlane((uint32_t)k);
    };
    bool more = true;  // a further tile may come (block-uniform)
    if (dyn && count == 0) grab_issue();
    // tile of step s, or false: none (the block's last grab, which found its pool empty)
    auto next = [&](uint32_t s, uint64_t& tile) __attribute__((always_inline)) {
      if (s < count) {
        tile = tile0 + s * tstep;
        if (dyn && s + 1 == count) grab_issue();  // the first dynamic tile, one step ahead
        return true;
      }
      if (!dyn) return false;
      const uint64_t k = grab_take();
      if (k >= per) return false;
      tile = pool0 + k;
      grab_issue();
      return true;
    };
    // Step s takes tile s-1 (loaded during step s-1), issues tile s, runs and stores tile s-1.
    // One issue site: the in-flight registers are a loop-carried value with an undefined entry,
    // so the register allocator has no phi copies to place (a copy before the wait would read
    // in-flight registers; tools/check_rq_isa.py checks the ISA for exactly that).
    uint64_t cur = 0;
    for (uint32_t s = 0;; ++s) {
      // younger than tile s-1's loads: tile s-2's stores (none before the second tile; at s = 0
      // nothing is in flight and take() reads registers nothing uses).  Unconditional, so every
      // path from an issue to the next read of its registers passes this wait.
      if constexpr (TWO)
        rq_vmwait_two<NLD>(s <= 1 ? 1u : 0u, pf_f, pf_b);
      else
        rq_vmwait_one<NLD>(s <= 1 ? 1u : 0u, pf_f);
      take();
      const uint64_t prev = cur;
      uint64_t tile = 0;
      if (more && next(s, tile)) {
        cur = tile_base(tile);
        issue(cur);
      } else {
        more = false;
      }
      if (s > 0) {
        run(xf, xb);
        store(xf, xb, prev);
      }
      if (!more) break;
    }
  }
  if constexpr (TWO) {
    __syncthreads();
    for (uint32_t i = t; i < fg.ngrad * FACC; i += NT) {
      const uint32_t k = i / FACC, e = i % FACC;
      real s = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) s += accw[w][k][e];
      reinterpret_cast<real*>(partials + (uint64_t)k * slot_stride + (uint64_t)blockIdx.x * RED)[e] = s;
    }
  }
}
template <bool TWO, int NT, bool PF>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PF ? QDC_RQ_PF_WAVES : 4)))
void k_rq(chunk* __restrict__ f, chunk* __restrict__ b, const fop* __restrict__ ops,
          const cx* __restrict__ mats, fgeo fg, uint32_t l0, cx* __restrict__ partials,
          uint64_t slot_stride) {
  rq_pass<TWO, NT, PF>(f, b, ops, mats, fg, l0, partials, slot_stride);
}

// One wave per tile (k_rw): the same programs, layouts and HBM addressing as k_rq with NT
// threads, run by one 64-lane wave.  Lane l holds the registers of k_rq's threads l + 64 e
// (e < NE = NT / 64) as its registers j + 16 e: k_rq's thread bits 6.. become register bits
// 4.. that no stage addresses (the host plan is unchanged).  What changes:
//  * a relayout is wave-local — LDS accesses of one wave execute in order, so it needs no
//    barrier (k_rq: two per relayout and state, coupling the tile's waves);
//  * every Gamma stage accumulates NE times the amplitudes per lane before its one 64-lane
//    reduce-scatter (the reduction's cost per amplitude divides by NE);
//  * waves are independent: while one computes, another on the SIMD loads or stores.
// Registers: R = 16 NE amplitudes per state and lane (two-state NE = 2: 128 VGPRs of tile),
// so 2 waves/SIMD.  One-state tiles (2^12 amplitudes) run on W = 2 waves with NE = 2 (a block
// of 128 threads holds k_rq's thread bits 0..6; relayouts then take block barriers).
#ifndef QDC_RW_WAVES
#define QDC_RW_WAVES 2
#endif
// one-state passes without prefetch (the f64 forward by default): 16 amplitudes per lane in f64
// need ~135 VGPRs, which 2 waves/SIMD would leave half idle
#ifndef QDC_RW_WAVES_HALF_ONE  // specialized one-state half-buffer passes (qdc_jit.hpp)
#define QDC_RW_WAVES_HALF_ONE 5
#endif
#ifndef QDC_RW_WAVES_ONE
#define QDC_RW_WAVES_ONE 2
#endif
// S5: five-slot layouts (NE = 2, W = 1): the register-group bit is register slot 4, which
// stages address like the other four, so covers hold 5 qubits (fewer relayouts); the layout
// descriptor then spans all 32 registers (rp[16 e + j], chunk offsets offi[8 e + i]).
// One-state forward passes on 2^12-amplitude tiles (round 3): W = 2, NE = 2, S5 and PF — two
// waves per tile, 32 amplitudes per lane, five register slots (k_rq's one-state tiles hold 16
// per thread: four slots, and a third of the forward's VALU time went to relayouts with their
// four-wave barriers), and the next tile's 16 chunks per lane prefetched into pinned VGPRs as in
// k_rq (rq_ld / rq_vmwait_two), with a dynamic tail taken block-wide.
// PROG (not void; non-prefetching instances): the pass program as straight-line stage calls
// (qdc_spec.hpp) in place of the interpreted op loop.
template <bool TWO, int NE, bool PF, int W, bool S5 = false, class PROG = void, bool HALF = false>
__device__ __forceinline__ void rw_pass(chunk* __restrict__ f, chunk* __restrict__ b,
                                        const fop* __restrict__ ops, const cx* __restrict__ mats,
                                        fgeo fg, uint32_t l0, cx* __restrict__ partials,
                                        uint64_t slot_stride) {
  static_assert(NE == 1 || NE == 2 || NE == 4, "k_rw: 1, 2 or 4 register groups");
  static_assert(!S5 || (NE == 2 && VEC == 2 && ((W == 1 && (!PF || !TWO)) || (W == 2 && PF && !TWO))),
                "five slots: f32 one-wave tiles, or the prefetching one-state tiles");
  static_assert(W == 1 || (W == 2 && !TWO), "k_rw: two-state tiles are one wave");
  constexpr int LOGNE = NE == 1 ? 0 : NE == 2 ? 1 : 2;
  constexpr int TB = W == 1 ? 6 : 7;  // k_rq thread bits held by the block's threads
  constexpr int R = RQ_R * NE;   // amplitudes per lane and state
  constexpr int CPT = R / VEC;   // chunks per lane and state
  constexpr int CPG = RQ_R / VEC;  // chunks per register group (f32 8, f64 16)
  // (HALF: a specialized one-wave program whose every relayout runs in two rounds through half
  // the buffer, qdc_spec.hpp spec_xchg_half)
  static_assert(!HALF || (W == 1 && !std::is_void<PROG>::value), "half buffers: one-wave programs");
  __shared__ cx buf[64 * W * R / (HALF ? 2 : 1)];
  __shared__ real accw[TWO ? FMAX_GRAD_RQ : 1][FACC];
  const uint32_t lane = threadIdx.x;  // the block's thread (W = 1: the lane)
  if constexpr (TWO) {
    for (uint32_t i = lane; i < FMAX_GRAD_RQ * FACC; i += 64) (&accw[0][0])[i] = 0;
  }
  const rqio* io = reinterpret_cast<const rqio*>(mats + l0 + sizeof(rq_layout) / sizeof(cx));
  uint64_t thr_ld = 0, thr_st = 0;  // this lane's chunk offsets in the load / store layout
#pragma unroll
  for (int k = 0; k < TB; ++k) {
    if ((lane >> k) & 1u) {
      thr_ld += io->gv_ld[k];
      thr_st += io->gv_st[k];
    }
  }
  // block-contiguous tiles (tile0 + s) or grid-strided (tile0 + s * grid: concurrently running
  // tiles are neighbours in memory)
  const bool gstride = fg.order == 1;  // 2: block-contiguous in XCD-aware block order
  const uint64_t tile0 = gstride ? (uint64_t)blockIdx.x
                                 : (uint64_t)xcd_block(blockIdx.x, gridDim.x, fg.order == 2) * fg.tpb;
  const uint64_t tstep = gstride ? (uint64_t)gridDim.x : 1u;
  // the static share: all tiles (ndyn = 0), or the block's tpb of the first nstat
  const uint64_t nst = (QDC_DYN_TAIL && fg_arg()->ndyn) ? fg_arg()->nstat : fg.ntiles;
  const uint32_t count =
      tile0 >= nst ? 0u
      : gstride    ? (uint32_t)((nst - 1 - tile0) / tstep + 1)
                   : (uint32_t)min<uint64_t>(fg.tpb, nst - tile0);
  // (geometry read through the kernarg pointer at each use: held in SGPRs across the pass it was
  // spilled to VGPR lanes and this ran on the VALU)
  auto tile_base = [&](uint64_t tile) {
    const fg_kptr a = fg_arg();
    uint64_t base = tile << a->lc;
    const uint32_t h = a->h;
#pragma unroll
    for (int k = 0; k < FMAX_ROWS; ++k)
      if ((uint32_t)k < h) base = insert_zero(base, a->hb[k]);
    return base + (base & a->gm);
  };
  auto rqio_now = [&]() {
    uint32_t ro = l0;
    asm volatile("" : "+s"(ro));
    return reinterpret_cast<const rqio*>(mats + ro + sizeof(rq_layout) / sizeof(cx));
  };
  // register group e (k_rq's thread bits 6.. = e): chunk offset sum of gv[6 + i] over e's bits
  auto goff = [&](const uint64_t* gv, int e) {
    uint64_t o = 0;
    if constexpr (S5) return o;  // slot 4 is a register chunk bit (offi)
#pragma unroll
    for (int i = 0; i < LOGNE; ++i)
      if ((e >> i) & 1) o += gv[TB + i];
    return o;
  };
  auto load = [&](cx (&xf)[R], cx (&xb)[R], uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    const chunk* pf = f + (base + thr_ld);
    const chunk* pb = b + (base + thr_ld);
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const uint64_t eo = goff(rg->gv_ld, e);
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const chunk cf = ldc(pf + (eo + rg->offi_ld[(S5 ? CPG * e : 0) + i]));
#pragma unroll
        for (int v = 0; v < VEC; ++v) xf[16 * e + VEC * i + v] = cf.v[v];
        if constexpr (TWO) {
          const chunk cb = ldc(pb + (eo + rg->offi_ld[(S5 ? CPG * e : 0) + i]));
#pragma unroll
          for (int v = 0; v < VEC; ++v) xb[16 * e + VEC * i + v] = cb.v[v];
        }
      }
    }
  };
  auto store = [&](cx (&xf)[R], cx (&xb)[R], uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    chunk* pf = f + (base + thr_st);
    chunk* pb = b + (base + thr_st);
    asm volatile("" : "+v"(pf), "+v"(pb));
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const uint64_t eo = goff(rg->gv_st, e);
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        chunk c;
#pragma unroll
        for (int v = 0; v < VEC; ++v) c.v[v] = xf[16 * e + VEC * i + v];
        stc(pf + (eo + rg->offi_st[(S5 ? CPG * e : 0) + i]), c);
        if constexpr (TWO) {
#pragma unroll
          for (int v = 0; v < VEC; ++v) c.v[v] = xb[16 * e + VEC * i + v];
          stc(pb + (eo + rg->offi_st[(S5 ? CPG * e : 0) + i]), c);
        }
      }
    }
  };
  // one state from layout Lc to Ln through the wave's LDS buffer: LDS operations of a wave
  // complete in issue order, so the reads see every lane's writes without a barrier, and the
  // next relayout's writes come after these reads
  // byte addressing: (a ^ b) * 8 = (a * 8) ^ (b * 8) with the uniform part scaled on the
  // scalar unit, so each access costs one v_xor (not an xor and a shift)
  char* const bufb = reinterpret_cast<char*>(buf);
  auto exchange = [&](cx (&x)[R], uint32_t tp, const rq_layout* Lc, uint32_t tpn,
                      const rq_layout* Ln) __attribute__((always_inline)) {
    uint32_t tpb = tp * (uint32_t)sizeof(cx), tpnb = tpn * (uint32_t)sizeof(cx);
    asm volatile("" : "+v"(tpb), "+v"(tpnb));  // opaque: LLVM would refactor the shift out
    if constexpr (W > 1) __syncthreads();  // the buffer's previous reads are done
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      uint32_t te = 0;
#pragma unroll
      for (int i = 0; i < LOGNE; ++i) te ^= (!S5 && ((e >> i) & 1)) ? Lc->tv[TB + i] : 0u;
#pragma unroll
      for (int j = 0; j < RQ_R; ++j) {
        const uint32_t u = (te ^ Lc->rp[(S5 ? 16 * e : 0) + j]) * (uint32_t)sizeof(cx);
        *reinterpret_cast<cx*>(__builtin_assume_aligned(bufb + (tpb ^ u), 8)) = x[16 * e + j];
      }
    }
    if constexpr (W > 1)
      __syncthreads();
    else
      __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      uint32_t te = 0;
#pragma unroll
      for (int i = 0; i < LOGNE; ++i) te ^= (!S5 && ((e >> i) & 1)) ? Ln->tv[TB + i] : 0u;
#pragma unroll
      for (int j = 0; j < RQ_R; ++j) {
        const uint32_t u = (te ^ Ln->rp[(S5 ? 16 * e : 0) + j]) * (uint32_t)sizeof(cx);
        x[16 * e + j] = *reinterpret_cast<const cx*>(__builtin_assume_aligned(bufb + (tpnb ^ u), 8));
      }
    }
    __builtin_amdgcn_wave_barrier();
  };
  auto run = [&](cx (&xf)[R], cx (&xb)[R]) __attribute__((always_inline)) {
    if constexpr (!std::is_same<PROG, void>::value) {
      static_assert(!PF || !TWO, "specialized k_rw passes: no two-state prefetching instance");
      const SpecEnv E{mats, ops, accw, lane, bufb};
      if constexpr (TWO)
        PROG{}(xf, xb, E);
      else
        PROG{}(xf, E);
      return;
    }
    uint32_t lcur = l0;
    uint32_t ri = 0;
    for (uint32_t j = 0; j < fg.nops; ++j) {
      const fop op = ops[j];
      const uint32_t kind = op.kind & 7u;
      const bool gamma = TWO && (op.kind & FOP_GAMMA) && !(QDC_RQ_ABL & 4);
      const cx* M = mats + op.mat;
      real* acc = TWO ? &accw[ri][0] : nullptr;
      if ((QDC_RQ_ABL & 2) && kind == FK_RELAYOUT) {
        lcur = op.mat;
        continue;
      }
      if ((QDC_RQ_ABL & 1) && kind != FK_RELAYOUT) {
        if (TWO && (op.kind & FOP_GAMMA)) ++ri;
        continue;
      }
      if (kind == FK_RELAYOUT) {
        const rq_layout* Lc = reinterpret_cast<const rq_layout*>(mats + lcur);
        const rq_layout* Ln = reinterpret_cast<const rq_layout*>(M);
        const uint32_t tp = rq_tp<TB>(Lc, lane), tpn = rq_tp<TB>(Ln, lane);
        exchange(xf, tp, Lc, tpn, Ln);
        if constexpr (TWO) exchange(xb, tp, Lc, tpn, Ln);
        lcur = op.mat;
        continue;
      }
      rq_stage<TWO>(kind * 64u + op.t1, xf, xb, M, gamma, acc);
      if (gamma) ++ri;
    }
  };
  // Gamma sums so far to dst[k * stride + e] (slot k), accumulators re-zeroed (dynamic tail)
  auto flush_acc = [&](cx* dst, uint64_t stride) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < fg.ngrad * FACC; i += 64) {
      const uint32_t k = i / FACC, e = i % FACC;
      reinterpret_cast<real*>(dst + (uint64_t)k * stride)[e] = accw[k][e];
      accw[k][e] = 0;
    }
    __builtin_amdgcn_wave_barrier();
  };
  cx xf[R], xb[R];  // xb unused (eliminated) in one-state passes
  if constexpr (!PF) {
    if (QDC_RQ_ABL & 32) {  // timing-only: no HBM traffic (registers start from the lane id)
#pragma unroll
      for (int j = 0; j < R; ++j) xf[j] = xb[j] = cx{(real)(lane + j) * 1e-3f, (real)j * 1e-3f};
    }
    auto tile = [&](uint64_t t) __attribute__((always_inline)) {
      const uint64_t base = tile_base(t);
      if (!(QDC_RQ_ABL & 32)) load(xf, xb, base);
      run(xf, xb);
      if (!(QDC_RQ_ABL & 32) || base == ~0ull) store(xf, xb, base);
    };
    // The static share, then (W = 1, fgeo::ndyn) the dynamic tail: this block's pool, one
    // granule of dgran tiles per grab.  The static tiles' Gamma sums are this block's partial,
    // each granule's go to its own (written when the next grab is due).  One loop, one call
    // site of the tile body (a second copy of it raised the spills).
    const bool dyn = QDC_DYN_TAIL && W == 1 && fg_arg()->ndyn != 0;
    const uint64_t per = dyn ? fg_arg()->ndyn / (8ull * fg_arg()->dgran) : 0;  // granules per pool
    uint32_t tt = 0, gleft = 0;
    uint64_t gi = ~0ull;  // current granule (~0: none yet)
    for (;;) {
      uint64_t t;
      if (tt < count) {
        t = tile0 + tt * tstep;
        ++tt;
      } else {
        if (!dyn) break;
        if (gleft == 0) {
          if constexpr (TWO) {
            if (gi == ~0ull)
              flush_acc(partials + (uint64_t)blockIdx.x * RED, slot_stride);
            else
              flush_acc(fg_arg()->dpart + gi * RED, fg_arg()->dstride);
          }
          const uint64_t k = fg_grab();
          if (k >= per) break;
          gi = (uint64_t)(blockIdx.x & 7u) * per + k;  // granule index in [0, ndyn / dgran)
          gleft = fg_arg()->dgran;
        }
        t = fg_arg()->nstat + gi * fg_arg()->dgran + (fg_arg()->dgran - gleft);
        --gleft;
      }
      tile(t);
    }
  } else if constexpr (!TWO) {
    // one-state prefetch (W = 1 or 2, NE = 2, S5): this lane's 16 chunks of the next tile in flight in
    // pinned v[192:255] while this tile runs; step s takes tile s-1, issues tile s, runs and
    // stores tile s-1 (k_rq's PF loop, with k_rw's register groups)
    static_assert(NE == 2 && (W == 1 || W == 2) && S5 && CPT == 16,
                  "one-state prefetch: S5 tiles of 2^11 (one wave) or 2^12 (two waves) amplitudes");
    constexpr int NLD = CPT;  // vector-memory ops per tile: loads = stores
    vec16 pf_a[8], pf_b[8];   // chunks 0..7 (register group 0) and 8..15 (group 1)
    auto issue = [&](uint64_t base) __attribute__((always_inline)) {
      const rqio* rg = rqio_now();
      const chunk* pfp = f + (base + thr_ld);
#define QDC_RW1_ISSUE(i)                                             \
  pf_a[i] = rq_ld<RQ_PIN_TWO + 4 * (i)>(pfp + rg->offi_ld[i]);       \
  pf_b[i] = rq_ld<RQ_PIN_TWO + 32 + 4 * (i)>(pfp + rg->offi_ld[8 + (i)]);
      QDC_RW1_ISSUE(0) QDC_RW1_ISSUE(1) QDC_RW1_ISSUE(2) QDC_RW1_ISSUE(3)
      QDC_RW1_ISSUE(4) QDC_RW1_ISSUE(5) QDC_RW1_ISSUE(6) QDC_RW1_ISSUE(7)
#undef QDC_RW1_ISSUE
    };
    auto take = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const chunk c = __builtin_bit_cast(chunk, pf_a[i]);
        const chunk d = __builtin_bit_cast(chunk, pf_b[i]);
        xf[2 * i] = c.v[0];
        xf[2 * i + 1] = c.v[1];
        xf[16 + 2 * i] = d.v[0];
        xf[16 + 2 * i + 1] = d.v[1];
      }
    };
    // dynamic tail, block-wide: thread 0 grabs step s+1's tile during step s (older than that
    // step's stores: the compiler's own wait for it is vmcnt(stores)), the block reads it from LDS
    __shared__ uint64_t grab_sh;
    unsigned long long grabbed = 0;
    const bool dyn = QDC_DYN_TAIL && fg_arg()->ndyn != 0;
    const uint64_t per = dyn ? fg_arg()->ndyn >> 3 : 0;
    auto grab_issue = [&]() __attribute__((always_inline)) {
      if (lane == 0) grabbed = atomicAdd(fg_arg()->dctr + FG_DCTR_STRIDE * (blockIdx.x & 7u), 1ull);
    };
    auto grab_take = [&]() __attribute__((always_inline)) {
      __syncthreads();
      if (lane == 0) grab_sh = (uint64_t)grabbed - fg_arg()->dbase;
      __syncthreads();
      const uint64_t k = grab_sh;
      return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(k >> 32)) << 32) |
             __builtin_amdgcn_readfirstlane((uint32_t)k);
    };
    if (dyn && count == 0) grab_issue();
    auto next = [&](uint32_t s, uint64_t& t) __attribute__((always_inline)) {
      if (s < count) {
        t = tile0 + s * tstep;
        if (dyn && s + 1 == count) grab_issue();
        return true;
      }
      if (!dyn) return false;
      const uint64_t k = grab_take();
      if (k >= per) return false;
      t = fg_arg()->nstat + (uint64_t)(blockIdx.x & 7u) * per + k;
      grab_issue();
      return true;
    };
    bool more = true;
    uint64_t cur = 0;
    for (uint32_t s = 0;; ++s) {
      rq_vmwait_two<NLD>(s <= 1 ? 1u : 0u, pf_a, pf_b);
      take();
      const uint64_t prev = cur;
      uint64_t t = 0;
      if (more && next(s, t)) {
        cur = tile_base(t);
        issue(cur);
      } else {
        more = false;
      }
      if (s > 0) {
        run(xf, xb);
        store(xf, xb, prev);
      }
      if (!more) break;
    }
  } else {
    static_assert(TWO && NE == 2, "k_rw prefetch: two-state tiles (32 chunks in a[0:127])");
    constexpr int NLD = 2 * CPT;  // vector-memory ops per tile: loads = stores
    vec16 pf[2 * CPT];            // chunk i of fwd at pf[i], of bwd at pf[CPT + i]
    auto issue = [&](uint64_t base) __attribute__((always_inline)) {
      const rqio* rg = rqio_now();
      const chunk* pfp = f + (base + thr_ld);
      const chunk* pbp = b + (base + thr_ld);
      const uint64_t e1 = rg->gv_ld[6];
#define QDC_RW_ISSUE(i)                                                                   \
  pf[i] = rw_lda<4 * (i)>(pfp + (((i) >= 8 ? e1 : 0) + rg->offi_ld[(i) & 7]));            \
  pf[CPT + (i)] = rw_lda<4 * (CPT + (i))>(pbp + (((i) >= 8 ? e1 : 0) + rg->offi_ld[(i) & 7]));
      QDC_RW_ISSUE(0) QDC_RW_ISSUE(1) QDC_RW_ISSUE(2) QDC_RW_ISSUE(3)
      QDC_RW_ISSUE(4) QDC_RW_ISSUE(5) QDC_RW_ISSUE(6) QDC_RW_ISSUE(7)
      QDC_RW_ISSUE(8) QDC_RW_ISSUE(9) QDC_RW_ISSUE(10) QDC_RW_ISSUE(11)
      QDC_RW_ISSUE(12) QDC_RW_ISSUE(13) QDC_RW_ISSUE(14) QDC_RW_ISSUE(15)
#undef QDC_RW_ISSUE
    };
    auto take = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {  // chunk i = register group i / 8, pair i % 8
        const chunk c = __builtin_bit_cast(chunk, pf[i]);
        const chunk d = __builtin_bit_cast(chunk, pf[CPT + i]);
        xf[2 * i] = c.v[0];
        xf[2 * i + 1] = c.v[1];
        xb[2 * i] = d.v[0];
        xb[2 * i + 1] = d.v[1];
      }
    };
    // as k_rq's PF loop: step s takes tile s-1, issues tile s, runs and stores tile s-1
    uint64_t cur = 0;
    for (uint32_t s = 0; s <= count; ++s) {
      rw_vmwait<NLD>(s <= 1 ? 1u : 0u, pf);
      take();
      const uint64_t prev = cur;
      if (s < count) {
        cur = tile_base(tile0 + s * tstep);
        issue(cur);
      }
      if (s > 0) {
        run(xf, xb);
        store(xf, xb, prev);
      }
    }
  }
  if constexpr (TWO) {
    // (a dynamic-tail pass wrote the block partial after its static tiles)
    if (PF || W != 1 || !QDC_DYN_TAIL || !fg_arg()->ndyn) {
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i = lane; i < fg.ngrad * FACC; i += 64) {
        const uint32_t k = i / FACC, e = i % FACC;
        reinterpret_cast<real*>(partials + (uint64_t)k * slot_stride + (uint64_t)blockIdx.x * RED)[e] =
            accw[k][e];
      }
    }
  }
}
template <bool TWO, int NE, bool PF, int W, bool S5 = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(
    (PF && TWO) ? 1 : (!TWO && !PF) ? QDC_RW_WAVES_ONE : QDC_RW_WAVES,
    (PF && TWO) ? 1 : (!TWO && !PF) ? QDC_RW_WAVES_ONE : QDC_RW_WAVES)))
void k_rw(chunk* __restrict__ f, chunk* __restrict__ b, const fop* __restrict__ ops,
          const cx* __restrict__ mats, fgeo fg, uint32_t l0, cx* __restrict__ partials,
          uint64_t slot_stride) {
  rw_pass<TWO, NE, PF, W, S5>(f, b, ops, mats, fg, l0, partials, slot_stride);
}

}  // namespace qdc
