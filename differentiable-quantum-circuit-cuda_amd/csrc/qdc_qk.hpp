// qdc_qk.hpp — dense k-qubit gates (k = 3..5) on MFMA (SURVEY.md §8 f rank 4; outside the
// reference's API, which stops at 2-qubit gates).
//
// A k-qubit gate maps each group of C = 2^k amplitudes (indices that differ only in the target
// bits) through a C×C complex matrix: out[r] = sum_c U[r*C + c] in[c], local index bit (k-1-b)
// = qubit pos[b] (pos[0] is the most significant, like q2gate's pos2, primitives.cu:573-620).
// In real form that is a 2C×2C matrix applied to 2^(n-k) vectors of 2C reals: a batched GEMM
// with 4C real MACs per amplitude (k=3: 32, k=5: 128), so at k >= 3 it is a real contraction
// and runs on the matrix cores: v_mfma_{f32,f64}_16x16x4 with the gate as the A operand
// (resident in VGPRs for the whole kernel) and 16 groups per instruction as the B operand.
//
// Operand mapping (16x16x4: A[i][kk] in lane kk*16 + i; B[kk][j] in lane kk*16 + j; D row i,
// column j in lane a*16 + j, register r, with i = 4a + r for f32 and i = 4r + a for f64).  Lane l = q*16 + j owns group j of the batch and
// its amplitudes c = (C/4) q + m, m < C/4 (both parts) — it loads them, and gets exactly them
// back in D, so the kernel is lane-local in place:
//   K step s (C/2 per output tile) reads B = part (s % 2) of amplitude (C/4) kk + s/2;
//   output tile t (C/8 of them): lane group a, register r = part (r % 2) of amplitude
//   (C/4) a + 2t + r/2 (qk_operands orders the gate's rows to match).
// The host forms each lane's A values (qk_operands) once per call.
#pragma once

#include "qdc_device.hpp"

namespace qdc {

constexpr int QK_MAX = 5;

struct qk_geo {
  uint64_t off[1 << QK_MAX];  // amplitude offset of local index c from the group base
  uint32_t sorted[QK_MAX];    // target positions, ascending (group base: insert zeros)
  uint32_t k;
  uint64_t ngroups;
};

// lane l's A operand for (tile t, K step s), at [(t * C/2 + s) * 64 + l]
template <int K>
inline void qk_operands(const cx* U, std::vector<real>& a) {
  constexpr int C = 1 << K;
  a.assign((size_t)(C / 8) * (C / 2) * 64, 0);
  for (int t = 0; t < C / 8; ++t)
    for (int s = 0; s < C / 2; ++s)
      for (int l = 0; l < 64; ++l) {
        const int i = l % 16, kk = l / 16;
        // D row i sits in lane group ga, register r: f32 i = 4 ga + r; f64 i = 4 r + ga
        // (probed: tools/mfma_layout_probe.hip, tools/mfma_f64_layout_probe.hip)
#ifdef QDC_F64
        const int ga = i % 4, r = i / 4;
#else
        const int ga = i / 4, r = i % 4;
#endif
        const int ro = (C / 4) * ga + 2 * t + r / 2, po = r % 2;
        const int ci = (C / 4) * kk + s / 2, pi = s % 2;
        const cx u = U[ro * C + ci];
        // [Re -Im; Im Re] acting on (re, im)
        const real v = po == 0 ? (pi == 0 ? u.x : -u.y) : (pi == 0 ? u.y : u.x);
        a[((size_t)t * (C / 2) + s) * 64 + l] = v;
      }
}

// P = 2 (f32, qubit 0 not a target): lane j of quad q owns the adjacent groups 2j and 2j + 1,
// whose amplitudes at each offset form one 16-B chunk — every load and store is 16 B per lane
// (256 contiguous bytes per quad) and each batch runs the MFMA chain twice.  P = 1: one group
// per lane, 8-B (f32) accesses.  PF: the next iteration's batches are loaded before this one's
// MFMA chains run (software pipelining: HBM latency hidden behind the matrix cores in every
// wave, not only across waves).
template <int K, int P, int NB, bool PF = false>
__global__ __launch_bounds__(256) void k_qk(cx* __restrict__ s, const real* __restrict__ aop,
                                            qk_geo g) {
  constexpr int C = 1 << K, T = C / 8, S = C / 2, M = C / 4;
#ifdef QDC_F64
  static_assert(P == 1, "f64 amplitudes are 16 B already");
  using acc_t = double __attribute__((ext_vector_type(4)));
#else
  using acc_t = float __attribute__((ext_vector_type(4)));
#endif
  const int l = threadIdx.x & 63;
  const int q = l >> 4, j = l & 15;
  real a[T][S];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int u = 0; u < S; ++u) a[t][u] = aop[((size_t)t * S + u) * 64 + l];
  uint64_t off[M];
#pragma unroll
  for (int m = 0; m < M; ++m) off[m] = g.off[M * q + m];
  // NB batches of 16 P groups per iteration, all loads first (bytes in flight per wave)
  constexpr uint64_t GB = 16 * P;  // groups per batch
  const uint64_t nbatch = (g.ngroups + GB - 1) / GB;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  struct batch {
    uint64_t base[NB];
    bool live[NB];
    cx x[NB][P][M];
  };
  auto load = [&](uint64_t bt0, batch& B) __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const uint64_t grp = (bt0 + nb) * GB + (uint64_t)j * P;
      B.live[nb] = grp < g.ngroups;  // ngroups is even when P = 2 (k < n)
      B.base[nb] = grp;
#pragma unroll
      for (int b = 0; b < K; ++b) B.base[nb] = insert_zero(B.base[nb], g.sorted[b]);
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if constexpr (P == 2) {
          const chunk c = B.live[nb] ? ldc(reinterpret_cast<const chunk*>(s + B.base[nb] + off[m]))
                                     : chunk{};
          B.x[nb][0][m] = c.v[0];
          B.x[nb][1][m] = c.v[1];
        } else {
          B.x[nb][0][m] = B.live[nb] ? s[B.base[nb] + off[m]] : cx{0, 0};
        }
      }
    }
  };
  auto apply_store = [&](const batch& B) __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        acc_t d[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          d[p] = acc_t{0, 0, 0, 0};
#pragma unroll
          for (int u = 0; u < S; ++u) {
            const real bv = (u & 1) ? B.x[nb][p][u >> 1].y : B.x[nb][p][u >> 1].x;
#ifdef QDC_F64
            d[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][u], bv, d[p], 0, 0, 0);
#else
            d[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][u], bv, d[p], 0, 0, 0);
#endif
          }
        }
        if (B.live[nb]) {
          if constexpr (P == 2) {
            chunk c0, c1;
            c0.v[0] = cx{d[0][0], d[0][1]};
            c0.v[1] = cx{d[1][0], d[1][1]};
            c1.v[0] = cx{d[0][2], d[0][3]};
            c1.v[1] = cx{d[1][2], d[1][3]};
            stc(reinterpret_cast<chunk*>(s + B.base[nb] + off[2 * t]), c0);
            stc(reinterpret_cast<chunk*>(s + B.base[nb] + off[2 * t + 1]), c1);
          } else {
            s[B.base[nb] + off[2 * t]] = cx{d[0][0], d[0][1]};
            s[B.base[nb] + off[2 * t + 1]] = cx{d[0][2], d[0][3]};
          }
        }
      }
    }
  };
  const uint64_t step = nwaves * NB;
  if constexpr (!PF) {
    for (uint64_t bt0 = wave * NB; bt0 < nbatch; bt0 += step) {
      batch B;
      load(bt0, B);
      apply_store(B);
    }
  } else {
    // two register sets, the loop unrolled by two so neither is copied
    batch B0, B1;
    uint64_t bt0 = wave * NB;
    if (bt0 < nbatch) load(bt0, B0);
    while (bt0 < nbatch) {
      if (bt0 + step < nbatch) load(bt0 + step, B1);
      apply_store(B0);
      bt0 += step;
      if (bt0 >= nbatch) break;
      if (bt0 + step < nbatch) load(bt0 + step, B0);
      apply_store(B1);
      bt0 += step;
    }
  }
}

// LDS-staged tiles (k_qkl), for gates with low target qubits.  k_qk's lanes j of a quad own 16
// consecutive groups, which are 16 consecutive chunks only when the low address bits are not
// targets: with targets among them every load instruction touches 64 lines for 16 B each
// (n = 28 f32, targets 1..5: 0.45 of HBM against 0.65 at 10..14, tools/qk_pos_probe.py).  Here a
// tile is 16 whole groups: the address bits below h (the four lowest non-target bits and the
// targets between them) plus every combination of the targets above h — 2^(k-L) contiguous
// chunks of 2^h amplitudes (L = targets below h).  A wave loads a tile with 16-B lane-contiguous
// accesses, stages it in LDS, each lane reads its MFMA operands (group j, amplitudes M q + m) and
// writes the results back to the cells it read, and the tile leaves as it came.
struct qkl_geo {
  uint64_t choff[1 << QK_MAX];  // amplitude offset of chunk c (bit i of c: target hi[i])
  uint32_t eoff[1 << QK_MAX];   // tile index of local amplitude ci in group 0
  uint32_t eg[16];              // tile index of group j's amplitude 0
  uint32_t hi[QK_MAX];          // targets >= h, ascending (tile base: insert zeros)
  uint32_t nhi, h;
  uint64_t ntiles;
};

// LDS cell of tile index e: XOR-swizzled within 256-B rows (16-B pieces stay whole), so the 16
// groups a quad reads at one amplitude — spread by the target bits between them — spread over
// the banks
__device__ __forceinline__ uint32_t qkl_swz(uint32_t e) {
  constexpr uint32_t PE = 256 / sizeof(cx);  // cells per 256-B row
  return e ^ (((e / PE) % (PE / VEC)) * VEC);
}

template <int K, int NB, bool PF = false>
__global__ __launch_bounds__(256) void k_qkl(cx* __restrict__ s, const real* __restrict__ aop,
                                             qkl_geo g) {
  constexpr int C = 1 << K, T = C / 8, S = C / 2, M = C / 4;
  constexpr int TA = 16 * C;          // amplitudes per tile
  constexpr int NP = TA / VEC / 64;   // 16-B pieces per lane per tile
  static_assert(NP >= 1, "tile smaller than one wave access");
#ifdef QDC_F64
  using acc_t = double __attribute__((ext_vector_type(4)));
#else
  using acc_t = float __attribute__((ext_vector_type(4)));
#endif
  __shared__ chunk lds[4][NB][TA / VEC];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = l >> 4, j = l & 15;
  real a[T][S];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int u = 0; u < S; ++u) a[t][u] = aop[((size_t)t * S + u) * 64 + l];
  uint32_t rd[M];  // this lane's operand cells
#pragma unroll
  for (int m = 0; m < M; ++m) rd[m] = qkl_swz(g.eoff[M * q + m] | g.eg[j]);
  uint32_t pc[NP];  // this lane's pieces: LDS chunk and amplitude offset from the tile base
  uint64_t po[NP];
  const uint32_t hmask = (1u << g.h) - 1u;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const uint32_t e = (uint32_t)(i * 64 + l) * VEC;
    pc[i] = qkl_swz(e) / VEC;
    po[i] = g.choff[e >> g.h] + (e & hmask);
  }
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  cx* cell = reinterpret_cast<cx*>(&lds[w][0][0]);
  uint64_t base[NB];
  chunk raw[NB][NP];
  auto load = [&](uint64_t t0) __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      base[nb] = (t0 + nb) << g.h;
      for (uint32_t b = 0; b < g.nhi; ++b) base[nb] = insert_zero(base[nb], g.hi[b]);
      if (t0 + nb < g.ntiles) {  // wave-uniform
#pragma unroll
        for (int i = 0; i < NP; ++i)
          raw[nb][i] = ldc(reinterpret_cast<const chunk*>(s + base[nb] + po[i]));
      }
    }
  };
  const uint64_t step = nwaves * NB;
  uint64_t t0 = wave * NB;
  if (t0 < g.ntiles) load(t0);
  while (t0 < g.ntiles) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < NP; ++i) lds[w][nb][pc[i]] = raw[nb][i];
    __builtin_amdgcn_wave_barrier();
    uint64_t cbase[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) cbase[nb] = base[nb];
    const uint64_t cur = t0;
    t0 += step;
    // PF: the staged tiles free the load registers, so the next tiles' loads are issued now and
    // fly while these run on the matrix cores
    if (PF && t0 < g.ntiles) load(t0);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      cx x[M];
#pragma unroll
      for (int m = 0; m < M; ++m) x[m] = cell[nb * TA + rd[m]];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        acc_t d = acc_t{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < S; ++u) {
          const real bv = (u & 1) ? x[u >> 1].y : x[u >> 1].x;
#ifdef QDC_F64
          d = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][u], bv, d, 0, 0, 0);
#else
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][u], bv, d, 0, 0, 0);
#endif
        }
        // outputs: amplitudes M q + 2t and M q + 2t + 1 of group j (qk_operands' row order)
        cell[nb * TA + rd[2 * t]] = cx{d[0], d[1]};
        cell[nb * TA + rd[2 * t + 1]] = cx{d[2], d[3]};
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      if (cur + nb < g.ntiles) {
#pragma unroll
        for (int i = 0; i < NP; ++i)
          stc(reinterpret_cast<chunk*>(s + cbase[nb] + po[i]), lds[w][nb][pc[i]]);
      }
    __builtin_amdgcn_wave_barrier();  // the next tiles overwrite these cells
    if (!PF && t0 < g.ntiles) load(t0);
  }
}

// k_qkl's geometry, or false when the state has fewer than four non-target qubits
inline bool qkl_plan(const size_t* pos, uint32_t k, uint32_t n, qkl_geo& g) {
  bool tgt[64] = {};
  for (uint32_t b = 0; b < k; ++b) tgt[pos[b]] = true;
  uint32_t h = 0, free = 0, gb[4];
  while (free < 4 && h < n) {
    if (!tgt[h]) gb[free++] = h;
    ++h;
  }
  if (free < 4) return false;
  g = qkl_geo{};
  g.h = h;
  int hidx[64];
  for (uint32_t p = h; p < n; ++p)
    if (tgt[p]) {
      hidx[p] = (int)g.nhi;
      g.hi[g.nhi++] = p;
    }
  for (uint32_t c = 0; c < (1u << g.nhi); ++c) {
    uint64_t o = 0;
    for (uint32_t i = 0; i < g.nhi; ++i)
      if ((c >> i) & 1u) o |= (uint64_t)1 << g.hi[i];
    g.choff[c] = o;
  }
  const uint32_t C = 1u << k;
  for (uint32_t ci = 0; ci < C; ++ci) {
    uint32_t lo = 0, c = 0;
    for (uint32_t b = 0; b < k; ++b) {
      if (!((ci >> (k - 1 - b)) & 1u)) continue;
      if (pos[b] < h) lo |= 1u << pos[b];
      else c |= 1u << hidx[pos[b]];
    }
    g.eoff[ci] = (c << h) | lo;
  }
  for (uint32_t jj = 0; jj < 16; ++jj) {
    uint32_t e = 0;
    for (int b = 0; b < 4; ++b)
      if ((jj >> b) & 1u) e |= 1u << gb[b];
    g.eg[jj] = e;
  }
  g.ntiles = (uint64_t)1 << (n - k - 4);
  return true;
}

}  // namespace qdc

namespace qdc {

// Operand uploads without host syncs: a ring of device slots, each with a pinned staging slot
// and an event recorded after the launch that reads it; a slot is rewritten only once that
// launch is done (hipEventSynchronize, which returns at once unless the GPU is QK_RING calls
// behind).
constexpr int QK_RING = 8;
struct QkRing {
  real* dev[QK_RING] = {};
  real* host[QK_RING] = {};
  hipEvent_t done[QK_RING] = {};
  size_t cap = 0;  // reals per slot
  int next = 0;
  const char* reserve(size_t n) {
    if (n <= cap) return nullptr;
    for (int i = 0; i < QK_RING; ++i) {
      if (done[i]) QDC_HIP(hipEventSynchronize(done[i]));
      if (dev[i]) QDC_HIP(hipFree(dev[i]));
      if (host[i]) QDC_HIP(hipHostFree(host[i]));
      dev[i] = nullptr;
      host[i] = nullptr;
      QDC_HIP(hipMalloc(&dev[i], n * sizeof(real)));
      QDC_HIP(hipHostMalloc(&host[i], n * sizeof(real)));
      if (!done[i]) QDC_HIP(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
    }
    cap = n;
    return nullptr;
  }
};

// Dense k-qubit gate on a state (k = 1, 2 route to the single-gate kernels).  `U` is the
// host gate (C×C row-major), `pos` the k target qubits (pos[0] most significant).  The
// operands go through the ring (read by the device before the host can touch the slot again).
inline const char* apply_qk(Ctx& c, cx* s, const qdc_complex* U, const size_t* pos, uint32_t k,
                            uint32_t n, QkRing& ring) {
  if (k == 1) return apply_dense<2>(c, s, to_mat<2>(U), (uint32_t)pos[0], (uint32_t)pos[0], n, "qk1");
  if (k == 2)
    return apply_dense<4>(c, s, to_mat<4>(U), (uint32_t)pos[0], (uint32_t)pos[1], n, "qk2");
  const uint32_t C = 1u << k;
  std::vector<cx> u(C * C);
  for (uint32_t i = 0; i < C * C; ++i) u[i] = cx{(real)U[i].re, (real)U[i].im};
  std::vector<real> a;
  if (k == 3) qk_operands<3>(u.data(), a);
  else if (k == 4) qk_operands<4>(u.data(), a);
  else qk_operands<5>(u.data(), a);
  qk_geo g{};
  g.k = k;
  g.ngroups = (uint64_t)1 << (n - k);
  for (uint32_t b = 0; b < k; ++b) g.sorted[b] = (uint32_t)pos[b];
  std::sort(g.sorted, g.sorted + k);
  for (uint32_t ci = 0; ci < C; ++ci) {
    uint64_t o = 0;
    for (uint32_t b = 0; b < k; ++b)
      if ((ci >> (k - 1 - b)) & 1u) o |= (uint64_t)1 << pos[b];
    g.off[ci] = o;
  }
  QDC_TRY(ring.reserve((size_t)(QK_MAX == 5 ? (32 / 8) * (32 / 2) * 64 : a.size())));
  const int slot = ring.next;
  ring.next = (ring.next + 1) % QK_RING;
  QDC_HIP(hipEventSynchronize(ring.done[slot]));  // the launch that last read this slot is done
  std::memcpy(ring.host[slot], a.data(), a.size() * sizeof(real));
  QDC_HIP(hipMemcpyAsync(ring.dev[slot], ring.host[slot], a.size() * sizeof(real),
                         hipMemcpyHostToDevice, c.stream));
  // 16-B accesses (two adjacent groups per lane) when qubit 0 is not a target (f32); measured
  // at n = 28 (tools/qk_probe.py): k = 3 +5-7 %, k = 5 +5 %, k = 4 -10 % (kept at 8 B)
  bool pair = sizeof(real) == 4 && g.sorted[0] != 0 && k != 4;
  if (const char* ev = getenv("QDC_QK_PAIR")) {
    const int v = atoi(ev);  // 0 off, 2: also at k = 4 (A/B)
    pair = v == 2 ? sizeof(real) == 4 && g.sorted[0] != 0 : pair && v != 0;
  }
  // batches per wave iteration (k_qk NB): 4 / 2 / 1 at k = 3 / 4 / 5, doubled ("wide": more
  // bytes in flight per wave) at k >= 4 — measured at n = 28 (tools/qk_probe.py,
  // profiles/r2o_qk_probe.log): k = 3 neutral, k = 4 +2 %, k = 5 +7 %.  Knob QDC_QK_WIDE=0/1
  const char* ew = getenv("QDC_QK_WIDE");
  bool wide = ew ? atoi(ew) != 0 : k >= 4;
  // software-pipelined batches (k_qk PF; knob QDC_QK_PF=0/1): NB batches in flight while the
  // previous NB run on the matrix cores — replaces "wide" (same registers).  Measured at n = 28
  // (tools/qk_probe.py --pf, profiles/r4i_qk_pf_ab.log): k = 3 0.643 -> 0.676, k = 5 0.515 ->
  // 0.562 of HBM, k = 4 0.573 -> 0.568; on by default at k = 3, 5.  With the doubled batches
  // (QDC_QK_PF=2, profiles/r4m_qk_ab.log): k = 3 0.676 -> 0.705, k = 4 0.577 -> 0.580, k = 5
  // 0.563 -> 0.549: the default at k = 3
  const char* epf = getenv("QDC_QK_PF");
  const int pfv = epf ? atoi(epf) : (k == 3 ? 2 : k == 5 ? 1 : 0);
  const bool pf = pfv != 0;
  const bool pfwide = pfv == 2;  // pipelined with the doubled batches (A/B)
  if (pf) wide = false;
  const uint64_t nb = (k == 3 ? 4 : k == 4 ? 2 : 1) * ((wide || pfwide) ? 2 : 1);
  const uint64_t gpb = pair ? 32 : 16;  // groups per batch
  const uint64_t waves = ((g.ngroups + gpb - 1) / gpb + nb - 1) / nb;
  uint32_t gmax = 256u * 16u;  // blocks (QDC_QK_GRID: another cap, A/B)
  if (const char* eg = getenv("QDC_QK_GRID")) gmax = (uint32_t)std::max(1, atoi(eg));
  const uint32_t grid = (uint32_t)std::min<uint64_t>((waves + 3) / 4, gmax);
  c.next_flops = 8.0 * C * (double)((uint64_t)1 << n);  // C complex MACs per amplitude
  const double bytes = 2.0 * state_bytes(n);
  const real* buf = ring.dev[slot];
  const char* e;
  // LDS-staged tiles when at least QDC_QK_LDS targets sit among the five lowest qubits (0:
  // never).  Measured at n = 28 f32 (tools/qk_pos_probe.py, profiles/r4w_qk_lds_ab.log): targets
  // 1..k 0.60 / 0.58 / 0.45 -> 0.68 / 0.67 / 0.63 of HBM at k = 3 / 4 / 5, bench.py's random
  // placements k = 4 0.58 -> 0.66, k = 5 0.57 -> 0.63; one low target at k = 3 is faster
  // through k_qk's paired groups (0.72 against 0.62), so k = 3 stages from two
  uint32_t nlow = 0;
  for (uint32_t b = 0; b < k; ++b) nlow += pos[b] < 5;
  int lds_min = k == 3 ? 2 : 1;
  if (const char* el = getenv("QDC_QK_LDS")) lds_min = atoi(el);
  qkl_geo lg;
  if (lds_min > 0 && (int)nlow >= lds_min && qkl_plan(pos, k, n, lg)) {
    // tiles per wave iteration: 8 KiB per wave in f32 at k >= 4
    constexpr bool f64 = sizeof(real) == 8;
    // QDC_QKL_VAR (A/B): 0 not pipelined, 1 pipelined, 2 pipelined with half the tiles at k = 5.
    // Same-box A/B (profiles/r4z_qkl_pf_ab.log, bench.py's placements, two repeats): k = 4
    // 0.648 / 0.640 -> 0.653 / 0.652, k = 5 0.617 / 0.612 -> 0.634 / 0.635 (2: 0.621 / 0.624),
    // k = 3 neutral
    int var = 1;
    if (const char* ev = getenv("QDC_QKL_VAR")) var = atoi(ev);
    const bool lpf = var != 0;
    const bool half5 = var == 2 || f64;
    const uint64_t nbl = k == 3 ? (f64 ? 2 : 4) : (k == 5 && half5) ? 1 : 2;
    const uint64_t lw = (lg.ntiles + nbl - 1) / nbl;
    const uint32_t lgrid = (uint32_t)std::min<uint64_t>((lw + 3) / 4, gmax);
#define QDC_QKL_LAUNCH(KK, NBB) \
  e = lpf ? c.launch_block("qk" #KK, bytes, k_qkl<KK, NBB, true>, lgrid, 256u, s, buf, lg) \
          : c.launch_block("qk" #KK, bytes, k_qkl<KK, NBB>, lgrid, 256u, s, buf, lg)
    if (k == 3) QDC_QKL_LAUNCH(3, f64 ? 2 : 4);
    else if (k == 4) QDC_QKL_LAUNCH(4, 2);
    else if (half5) QDC_QKL_LAUNCH(5, 1);
    else QDC_QKL_LAUNCH(5, 2);
#undef QDC_QKL_LAUNCH
    QDC_TRY(e);
    QDC_HIP(hipEventRecord(ring.done[slot], c.stream));
    return nullptr;
  }
#define QDC_QK_LAUNCH(KK, PP, NB3)                                                              \
  e = pfwide ? c.launch_block("qk" #KK, bytes, k_qk<KK, PP, 2 * (NB3), true>, grid, 256u, s, buf, g) \
      : pf   ? c.launch_block("qk" #KK, bytes, k_qk<KK, PP, (NB3), true>, grid, 256u, s, buf, g) \
      : wide ? c.launch_block("qk" #KK, bytes, k_qk<KK, PP, 2 * (NB3)>, grid, 256u, s, buf, g)   \
             : c.launch_block("qk" #KK, bytes, k_qk<KK, PP, (NB3)>, grid, 256u, s, buf, g)
#ifndef QDC_F64
  if (pair) {
    if (k == 3) QDC_QK_LAUNCH(3, 2, 4);
    else if (k == 4) QDC_QK_LAUNCH(4, 2, 2);
    else QDC_QK_LAUNCH(5, 2, 1);
  } else
#endif
  if (k == 3) QDC_QK_LAUNCH(3, 1, 4);
  else if (k == 4) QDC_QK_LAUNCH(4, 1, 2);
  else QDC_QK_LAUNCH(5, 1, 1);
#undef QDC_QK_LAUNCH
  QDC_TRY(e);
  QDC_HIP(hipEventRecord(ring.done[slot], c.stream));
  return nullptr;
}

}  // namespace qdc
