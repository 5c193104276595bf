// qdc_spec.hpp — reverse-sweep passes specialized per pass program (round 3).
//
// The generic two-state kernel (k_rw<true, 2, false, 1, true>) interprets a pass program: per
// op it loads a descriptor, branches over ~25 slot cases and runs one stage.  Measured on the
// committed library: its register allocation keeps every stage's outputs
// apart from the loop-carried state and copies 63 register pairs back at the end of each stage
// (plus one spilled pair through scratch), ~6.5 % of the pass's VALU instructions, and every
// stage waits on a dependent scalar-load chain (op descriptor, then matrix).  A pass written
// out as straight-line code has no loop-carried state across stages, so none of that exists:
// the same stage templates (qdc_rq.hpp), the same HBM addressing, the same dynamic tail and Γ
// partials — bit-identical results — with each stage's slot case, Γ flag and every relayout's
// LDS descriptors compile-time constants.  The host (qdc_jit.hpp) writes one such kernel per
// distinct pass program, compiles it with hipcc for gfx950 on first use and caches the code
// object.
#pragma once

#include "qdc_rq.hpp"

namespace qdc {

struct SpecEnv {
  const cx* mats;
  const fop* ops;
  real (*accw)[FACC];
  uint32_t lane;
  char* bufb;
};

// one state from layout c to layout n through the wave's LDS buffer, the descriptors constants
__device__ __forceinline__ void spec_xchg(cx (&x)[32], const SpecEnv& E, const uint32_t* rpc,
                                          const uint32_t* tvc, const uint32_t* rpn,
                                          const uint32_t* tvn) {
  uint32_t tp = 0, tpn = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    tp ^= ((E.lane >> k) & 1u) ? tvc[k] : 0u;
    tpn ^= ((E.lane >> k) & 1u) ? tvn[k] : 0u;
  }
  uint32_t tpb = tp * (uint32_t)sizeof(cx), tpnb = tpn * (uint32_t)sizeof(cx);
  asm volatile("" : "+v"(tpb), "+v"(tpnb));
#pragma unroll
  for (int j = 0; j < 32; ++j)
    *reinterpret_cast<cx*>(__builtin_assume_aligned(E.bufb + (tpb ^ (rpc[j] * (uint32_t)sizeof(cx))), 8)) = x[j];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 32; ++j)
    x[j] = *reinterpret_cast<const cx*>(
        __builtin_assume_aligned(E.bufb + (tpnb ^ (rpn[j] * (uint32_t)sizeof(cx))), 8));
  __builtin_amdgcn_wave_barrier();
}

// The tile loop of k_rw<true, 2, false, 1, true> (f32, one wave per 2^11-amplitude two-state
// tile, five register slots) with the pass program PROG (a functor written by the host) in
// place of the interpreted op loop.  Everything else is k_rw's code path: static shares, the
// per-XCD dynamic tail with granule partials, Γ accumulators in LDS, the block partials.
template <class PROG>
__device__ __forceinline__ void rw_spec_two(chunk* __restrict__ f, chunk* __restrict__ b,
                                            const fop* __restrict__ ops,
                                            const cx* __restrict__ mats, fgeo fg, uint32_t l0,
                                            cx* __restrict__ partials, uint64_t slot_stride) {
  static_assert(VEC == 2, "specialized reverse passes: f32");
  constexpr int R = 32, CPG = RQ_R / VEC;
  __shared__ cx buf[64 * R];
  __shared__ real accw[FMAX_GRAD_RQ][FACC];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < FMAX_GRAD_RQ * FACC; i += 64) (&accw[0][0])[i] = 0;
  const rqio* io = reinterpret_cast<const rqio*>(mats + l0 + sizeof(rq_layout) / sizeof(cx));
  uint64_t thr_ld = 0, thr_st = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    if ((lane >> k) & 1u) {
      thr_ld += io->gv_ld[k];
      thr_st += io->gv_st[k];
    }
  }
  const bool gstride = fg.order == 1;
  const uint64_t tile0 = gstride ? (uint64_t)blockIdx.x
                                 : (uint64_t)xcd_block(blockIdx.x, gridDim.x, fg.order == 2) * fg.tpb;
  const uint64_t tstep = gstride ? (uint64_t)gridDim.x : 1u;
  const uint64_t nst = (QDC_DYN_TAIL && fg_arg()->ndyn) ? fg_arg()->nstat : fg.ntiles;
  const uint32_t count =
      tile0 >= nst ? 0u
      : gstride    ? (uint32_t)((nst - 1 - tile0) / tstep + 1)
                   : (uint32_t)min<uint64_t>(fg.tpb, nst - tile0);
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
  cx xf[R], xb[R];
  auto load = [&](uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    const chunk* pf = f + (base + thr_ld);
    const chunk* pb = b + (base + thr_ld);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const chunk cf = ldc(pf + rg->offi_ld[CPG * e + i]);
        const chunk cb = ldc(pb + rg->offi_ld[CPG * e + i]);
        xf[16 * e + 2 * i] = cf.v[0];
        xf[16 * e + 2 * i + 1] = cf.v[1];
        xb[16 * e + 2 * i] = cb.v[0];
        xb[16 * e + 2 * i + 1] = cb.v[1];
      }
  };
  auto store = [&](uint64_t base) __attribute__((always_inline)) {
    const rqio* rg = rqio_now();
    chunk* pf = f + (base + thr_st);
    chunk* pb = b + (base + thr_st);
    asm volatile("" : "+v"(pf), "+v"(pb));
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        chunk c;
        c.v[0] = xf[16 * e + 2 * i];
        c.v[1] = xf[16 * e + 2 * i + 1];
        stc(pf + rg->offi_st[CPG * e + i], c);
        c.v[0] = xb[16 * e + 2 * i];
        c.v[1] = xb[16 * e + 2 * i + 1];
        stc(pb + rg->offi_st[CPG * e + i], c);
      }
  };
  const SpecEnv E{mats, ops, accw, lane, reinterpret_cast<char*>(buf)};
  auto flush_acc = [&](cx* dst, uint64_t stride) __attribute__((always_inline)) {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < fg.ngrad * FACC; i += 64) {
      const uint32_t k = i / FACC, e = i % FACC;
      reinterpret_cast<real*>(dst + (uint64_t)k * stride)[e] = accw[k][e];
      accw[k][e] = 0;
    }
    __builtin_amdgcn_wave_barrier();
  };
  const bool dyn = QDC_DYN_TAIL && fg_arg()->ndyn != 0;
  const uint64_t per = dyn ? fg_arg()->ndyn / (8ull * fg_arg()->dgran) : 0;
  uint32_t tt = 0, gleft = 0;
  uint64_t gi = ~0ull;
  for (;;) {
    uint64_t t;
    if (tt < count) {
      t = tile0 + tt * tstep;
      ++tt;
    } else {
      if (!dyn) break;
      if (gleft == 0) {
        if (gi == ~0ull)
          flush_acc(partials + (uint64_t)blockIdx.x * RED, slot_stride);
        else
          flush_acc(fg_arg()->dpart + gi * RED, fg_arg()->dstride);
        const uint64_t k = fg_grab();
        if (k >= per) break;
        gi = (uint64_t)(blockIdx.x & 7u) * per + k;
        gleft = fg_arg()->dgran;
      }
      t = fg_arg()->nstat + gi * fg_arg()->dgran + (fg_arg()->dgran - gleft);
      --gleft;
    }
    const uint64_t base = tile_base(t);
    load(base);
    PROG{}(xf, xb, E);
    store(base);
  }
  if (!QDC_DYN_TAIL || !fg_arg()->ndyn) {
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < fg.ngrad * FACC; i += 64) {
      const uint32_t k = i / FACC, e = i % FACC;
      reinterpret_cast<real*>(partials + (uint64_t)k * slot_stride + (uint64_t)blockIdx.x * RED)[e] =
          accw[k][e];
    }
  }
}

}  // namespace qdc
