// qdc_spec.hpp — register-resident passes specialized per pass program (round 3).
//
// The generic register-resident kernels (k_rw, k_rq: qdc_rq.hpp) interpret a pass program: per
// op they load a descriptor, branch over ~25 slot cases and run one stage.  Measured on the
// two-state f32 kernel: its register allocation keeps every stage's
// outputs apart from the loop-carried state and copies 63 register pairs back at the end of
// each stage (plus one spilled pair through scratch), ~6.5 % of the pass's VALU instructions,
// and every stage waits on a dependent scalar-load chain (op descriptor, then matrix).  A pass
// written out as straight-line code has no loop-carried state across stages, so none of that
// exists: the same stage templates, the same HBM addressing, the same dynamic tail and Γ
// partials (the kernels' own code: rw_pass / rq_pass with the program as a functor) —
// bit-identical results — with each stage's slot case, Γ flag and every relayout's LDS
// descriptors compile-time constants.  The host (qdc_jit.hpp) writes one such kernel per
// distinct pass program, compiles it with hipcc for gfx950 on first use and caches the code
// object.  Instances: f32 two-state five-slot reverse passes (k_rw<true, 2, false, 1, true>),
// f32 one-state forward passes (k_rq<false, 256, true>), f64 two-state reverse passes
// (k_rw<true, 1, false, 1>) and f64 one-state passes (k_rw<false, 1, false, W>).
#pragma once

#include "qdc_rq.hpp"

namespace qdc {

// One state from layout c to layout n through the block's LDS buffer, the descriptors
// constants (the interpreted kernels' XOR addressing: one v_xor per access).  TB thread bits;
// BAR: the tile spans several waves (block barriers, as rq_exchange), else one wave (LDS
// operations of a wave complete in order: wave barriers only keep the compiler's order).
template <int TB, bool BAR, int R>
__device__ __forceinline__ void spec_xchg(cx (&x)[R], const SpecEnv& E, const uint32_t* rpc,
                                          const uint32_t* tvc, const uint32_t* rpn,
                                          const uint32_t* tvn) {
  uint32_t tp = 0, tpn = 0;
#pragma unroll
  for (int k = 0; k < TB; ++k) {
    tp ^= ((E.t >> k) & 1u) ? tvc[k] : 0u;
    tpn ^= ((E.t >> k) & 1u) ? tvn[k] : 0u;
  }
  uint32_t tpb = tp * (uint32_t)sizeof(cx), tpnb = tpn * (uint32_t)sizeof(cx);
  asm volatile("" : "+v"(tpb), "+v"(tpnb));
  if constexpr (BAR) __syncthreads();
#pragma unroll
  for (int j = 0; j < R; ++j)
    *reinterpret_cast<cx*>(__builtin_assume_aligned(E.bufb + (tpb ^ (rpc[j] * (uint32_t)sizeof(cx))), 8)) = x[j];
  if constexpr (BAR)
    __syncthreads();
  else
    __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < R; ++j)
    x[j] = *reinterpret_cast<const cx*>(
        __builtin_assume_aligned(E.bufb + (tpnb ^ (rpn[j] * (uint32_t)sizeof(cx))), 8));
  if constexpr (!BAR) __builtin_amdgcn_wave_barrier();
}

// One-wave exchange through half the buffer: a tile bit that both layouts hold in the same
// register slot S splits it into two rounds, each moving the registers with slot bit S = p
// through an LDS index without that bit (rpc / rpn / tvc / tvn are formed on the compressed
// index, qdc_jit.hpp).  A round writes and reads the same registers, so nothing is overwritten
// before it is written; the kernel then needs 2^(T-1) * 8 B of LDS per wave instead of 2^T * 8
// (one-state five-slot tiles: 8 KiB, so LDS no longer caps them at 2.5 waves per SIMD).
template <int TB, int R, int S>
__device__ __forceinline__ void spec_xchg_half(cx (&x)[R], const SpecEnv& E, const uint32_t* rpc,
                                               const uint32_t* tvc, const uint32_t* rpn,
                                               const uint32_t* tvn) {
  uint32_t tp = 0, tpn = 0;
#pragma unroll
  for (int k = 0; k < TB; ++k) {
    tp ^= ((E.t >> k) & 1u) ? tvc[k] : 0u;
    tpn ^= ((E.t >> k) & 1u) ? tvn[k] : 0u;
  }
  uint32_t tpb = tp * (uint32_t)sizeof(cx), tpnb = tpn * (uint32_t)sizeof(cx);
  asm volatile("" : "+v"(tpb), "+v"(tpnb));
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (((j >> S) & 1) == p)
        *reinterpret_cast<cx*>(__builtin_assume_aligned(E.bufb + (tpb ^ (rpc[j] * (uint32_t)sizeof(cx))), 8)) = x[j];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (((j >> S) & 1) == p)
        x[j] = *reinterpret_cast<const cx*>(
            __builtin_assume_aligned(E.bufb + (tpnb ^ (rpn[j] * (uint32_t)sizeof(cx))), 8));
    __builtin_amdgcn_wave_barrier();
  }
}

// The same exchange with LDS addresses that need no VALU per access: the LDS index is a bit
// permutation of the tile index that puts the current layout's thread bits on index bits
// 0..TB-1 and its register slots above, so every write goes to t * sizeof(cx) + j * 2^TB *
// sizeof(cx) bytes (a per-thread constant plus an immediate offset), and every read to a
// per-thread part (the new layout's thread bits, permuted: pn) plus the register's immediate
// offset offr[j] (its slot bits, permuted).  The two parts of a read address are disjoint bits,
// so they add.
template <int TB, bool BAR, int R>
__device__ __forceinline__ void spec_xchg_imm(cx (&x)[R], const SpecEnv& E, const uint32_t* pn,
                                              const uint32_t* offr) {
  uint32_t rb = 0;
#pragma unroll
  for (int k = 0; k < TB; ++k) rb |= ((E.t >> k) & 1u) ? pn[k] : 0u;
  uint32_t wb = E.t * (uint32_t)sizeof(cx);
  asm volatile("" : "+v"(rb), "+v"(wb));
  if constexpr (BAR) __syncthreads();
#pragma unroll
  for (int j = 0; j < R; ++j)
    *reinterpret_cast<cx*>(__builtin_assume_aligned(
        E.bufb + wb + (uint32_t)j * (1u << TB) * (uint32_t)sizeof(cx), 8)) = x[j];
  if constexpr (BAR)
    __syncthreads();
  else
    __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < R; ++j)
    x[j] = *reinterpret_cast<const cx*>(__builtin_assume_aligned(E.bufb + rb + offr[j], 8));
  if constexpr (!BAR) __builtin_amdgcn_wave_barrier();
}

}  // namespace qdc
