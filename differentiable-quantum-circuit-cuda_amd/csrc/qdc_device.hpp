// qdc_device.hpp — host-side launch layer: per-stream context, partial-sum arena,
// launch geometry, per-kernel event profiling, host small-matrix algebra.
//
// Replaces the reference's per-call host plumbing (src/primitives.cu:114-138 cuBLAS
// handle per inverse, :255-292 malloc/launch/D2H/host-sum/free per reduction) with one
// context per stream that owns every scratch buffer for its lifetime.
#pragma once

#include <atomic>

#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "qdc/primitives.h"
#include "qdc_kernels.hpp"

namespace qdc {

static_assert(sizeof(cx) == sizeof(qdc_complex), "complex layout");

// ---------------------------------------------------------------------------------------
// Errors: NULL = ok, else a message in thread-local storage (the caller never frees it;
// the reference leaks a malloc'd string instead, primitives.cu:37-47).
// ---------------------------------------------------------------------------------------
inline const char* fail(const char* fmt, ...) {
  static thread_local char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return buf;
}

#define QDC_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t qdc_e_ = (call);                                                        \
    if (qdc_e_ != hipSuccess)                                                          \
      return ::qdc::fail("HIP ERROR: call of a function \"%s\" in line %d of file %s " \
                         "failed with %s.",                                            \
                         #call, __LINE__, __FILE__, hipGetErrorName(qdc_e_));          \
  } while (0)

#define QDC_TRY(expr)                  \
  do {                                 \
    const char* qdc_m_ = (expr);       \
    if (qdc_m_ != nullptr) return qdc_m_; \
  } while (0)

// ---------------------------------------------------------------------------------------
// Profiling: optional start/stop events around every launch of a context's stream.
// Used by bench.py to measure each kernel's average duration inside the timed region.
// ---------------------------------------------------------------------------------------
struct ProfRecord {
  const char* name;
  double bytes;
  double flops;
  hipEvent_t a, b;
};

struct Prof {
  bool on = false;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<ProfRecord> recs;
  // Timing-only events: no system-scope fence when an event is recorded (a default event writes
  // back and invalidates the caches at every record, i.e. twice per profiled launch, and the
  // next kernel starts cold).  The records are read only after the stream is synchronised.
  // QDC_EVENT_FENCE=1 restores default events.
  unsigned flags = hipEventDisableSystemFence;

  hipEvent_t get() {
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[used++];
  }
  void reset() {
    used = 0;
    recs.clear();
  }
  ~Prof() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

// ---------------------------------------------------------------------------------------
// Context: one HIP stream + the scratch it needs.  Every op of a context is ordered on its
// stream; host-visible results synchronise that stream only.
// ---------------------------------------------------------------------------------------
constexpr uint32_t NBMAX = 4096;  // max blocks of a reduction launch = partials per slot

// Restores the caller's current HIP device on every return path of a C-ABI entry point: a
// multi-device circuit switches devices per shard (Ctx::use), and the primitives, torch and
// the caller's own code must not find themselves on the last shard's GPU afterwards.
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (dev >= 0 && (hipGetDevice(&cur) != hipSuccess || cur != dev)) (void)hipSetDevice(dev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t grid_cap = 1u << 20;  // streaming launches: ~one item per thread (measured best)
  uint32_t red_cap = 2048;   // target blocks of reduction launches (<= NBMAX)
  // the same for the single-gate reverse with its gradient (both states read and written; knob
  // QDC_REV_RED): at 4096 instead of 2048 blocks reverse_q2 +1..2 points at 5 of 7 pairs
  // ((26,27) 72.4 -> 74.3 %, (0,1) 75.9 -> 77.1 %), reverse_q1 +0.5..1 (profiles/r6/r6m)
  uint32_t rev_red_cap = NBMAX;
  double next_flops = 0;     // algorithmic FLOPs of the next launch (profiling; reset by launch)
  // gap mask of the states this context's gate-shaped launches address: chunk c of a state at
  // c + (c & gm).  Nonzero for a circuit whose fwd / bwd states are interleaved in one
  // allocation (qdc_circuit.hpp alloc_pair); 0 (plain) for the primitives' states.
  uint64_t gm = 0;
  // minimum items per thread of streaming (non-reducing) direct / diagonal launches (knob
  // QDC_DIRECT_IT; 0: one item per thread).  tools/pair_probe.hip streams a far q1 pair at
  // 5.3 / 5.55 / 5.9 TB/s with 1 / 2 / 4 items per thread in flight
  uint32_t direct_it = 0;
  // gates with no target at chunk bit 0..5 run on the TILE family too (far targets as row
  // bits) instead of the direct rows.  Knob QDC_TILE_FAR, one bit per op class: bit 0 reverse
  // (both states read and written), bit 1 one-state ops, bit 2 inject / grad.  Measured at
  // n = 28 (profiles/r2m_micro_table_tf*.txt): reverse_q1 68-70 -> 75-77 % of 8 TB/s at every
  // far position; one-state ops were slower tiled on 2^10 / 2^11-chunk tiles (apply 77 -> 68 %
  // at some positions), but on 2^12-chunk tiles (tile1_wide = 2) they lift the positions the
  // direct rows lose (apply_q1 at 20 / 24 69.9 / 69.2 -> 71.6 / 71.5 %, apply_q2 (5,20) 68.0 ->
  // 70.8 %, profiles/r4k_micro_tune.log): bits 0 and 1 on
  uint32_t tile_far = 3;
  // XCD-aware block order of streaming single-gate launches (direct and tile families; knob
  // QDC_XCD_MAP): the blocks one XCD runs own adjacent ranges.  Measured at n = 28
  // (profiles/r2t_micro_table_xcd*.txt): injections at q1 1..6 71 -> 76 %, apply/inject at
  // q1 7..11 and 21..23 +4..7 points, apply_q2 71.6 -> 73.4 %; q1 24 71.8 -> 69.4 %.
  // Bits: 0 streaming launches, 1 reducing launches, 2 diagonal launches (k_diag, round 6)
  uint32_t xcd_map = 1;
  // two-state tile-family launches on 2^10-chunk tiles (K = 4, 32 KiB of LDS per block) instead
  // of 2^9 (knob QDC_TILE2_WIDE): longer rows per far row bit.  Measured at n = 28
  // (profiles/r2y_micro_table_tile2_wide*.txt): reverse_q2 +1.2..3.3 points on every pair
  // ((26,27) 66.3 -> 69.6 %, (14,13) 69.4 -> 71.4 %), reverse_q1 and injections within +-0.5
  // (round 4: 2^11-chunk two-state tiles, 64 KiB of LDS: reverse_q2 (26,27) 69.4 -> 72.3 %,
  // (14,13) 71.3 -> 73.8 %, reverse_q1 75.8 -> 77.5-78 %, profiles/r4k_micro_tune.log)
  uint32_t tile2_wide = 2;
  // one-state tile-family launches on 2^(10 + tile1_wide)-chunk tiles (1: K = 8, 32 KiB of LDS;
  // 2: K = 16, 64 KiB; knob QDC_TILE1_WIDE)
  uint32_t tile1_wide = 2;
  // single-gate ops on the LANE family (k_lane: one chunk per lane, partners across lanes;
  // knob QDC_LANE, one bit per op class: bit 0 reverse, bit 1 streaming one-state ops and
  // injections, bit 2 densities and gradients).  Measured at n = 28 f32 (profiles/r5/
  // r5k_*, r5l_*): apply 72-74 -> 76-84 % of 8 TB/s at most placements; the reverse with its
  // gradient 77.5 -> 65-67 % at far targets (the tile family's 32 KiB runs per state win for
  // two states), densities within +-1: bit 1 only
  uint32_t lane_ops = 2;
  // units in flight per wave of LANE launches, per class as lane_ops (knob QDC_LANE_U="u0,u1,u2";
  // 1, 4 or 8)
  uint32_t lane_u[3] = {8, 1, 4};
  // chunks per state in flight per thread and step of the diagonal reverse kernels (knob
  // QDC_DIAG_RU: 4, 8 or 16; k_diag takes 2 or 8; 8 = a block's step moves 32 KiB of each state,
  // as the tile family): k_diag reverse_q2_diag 71.4 -> 73.3 % (profiles/r5/r5l_*); k_diag_q
  // 74.5 / 75.4 / 76.7 % at 4 / 8 / 16 (profiles/r6/r6l)
  uint32_t diag_ru = 16;
  // target blocks of the diagonal reverse's reducing launches (knob QDC_DIAG_RED, <= NBMAX):
  // k_diag_q with 16 in flight 76.7 -> 77.3 % at 2048 -> 4096 blocks (profiles/r6/r6l)
  uint32_t diag_red = NBMAX;
  // diagonal reverse launches on k_diag_q (k and the matrix entries fixed per thread; knob
  // QDC_DIAG_Q = 0: k_diag)
  uint32_t diag_q = 1;
  // tile-family blocks of several tiles (reducing launches) load the next tile during this
  // tile's math (knob QDC_TILE_PF), on tiles without far row bits: reverse_q2 (0,1) / (1,2)
  // +0.7..1.0 points; with row bits it measured 2.5-3 points slower (reverse_q1 at 12..27,
  // reverse_q2 (5,20), (27,0); profiles/r6/r6m)
  uint32_t tile_pf = 1;
  // streaming LANE launches with a target beyond the wave's chunk bits on the block-wide
  // variant (k_lane_blk; knob QDC_LANE_BLK): +1..3.5 points at 13 of 27 far placements, -1..4
  // at 5 (profiles/r5/r5m_*, r5n_*); the far-row cells that stay near 71 % (q1 20, 24) do so
  // under every variant and block order tried: a DRAM-mapping effect of the row distance
  // (tools/r5/stream_probe2.hip: plain two-row streams at chunk bit 20 reach 72.6 %)
  uint32_t lane_blk = 1;
  // Address-map exceptions of the one-state application (f32 n = 28 sweep, every q1 position
  // and 8 q2 pairs, LANE vs its wave variant vs the tile family, two repeats on one box:
  // profiles/r6/r6v), keyed by the byte stride 2^b of a target (b = position + 3 in f32, + 4 in
  // f64).  The tile family streams every far q1 at a flat 73 %; LANE beats it everywhere except
  // at b = 23 and 27 (q1 20 / 24: 72.0 / 71.5 %), where the pair's two rows collide in the
  // DRAM map: those run on the tile family (knob QDC_LANE_TILE_BITS, a mask of b).  The wave
  // variant of LANE beats the block-wide one at b = 15 (q1 12: 80.7 -> 85.0 %) and 23 (q2
  // (5,20): 72.8 -> 75.0 %) and loses 1-3 points at 9 other placements (knob
  // QDC_LANE_NOBLK_BITS).
  uint64_t lane_tile_bits = (1ull << 23) | (1ull << 27);
  uint64_t lane_noblk_bits = (1ull << 15) | (1ull << 23);
  // reduction arena
  cx* partials = nullptr;  // [FIN_MAX][NBMAX][RED]
  cx* results = nullptr;   // [FIN_MAX][RED] scratch destination for one-shot reductions
  cx* host_results = nullptr;  // pinned [FIN_MAX][RED]
  std::vector<cx*> pending_dst;  // destinations (a slot of some reduction base)
  std::vector<uint32_t> pending_nb;
  cx* pending_base = nullptr;
  int pending_accumulate = 0;
  Prof prof;
  unsigned long long* dctr = nullptr;  // 8 dynamic-tail counters (plan_dyn)
  uint64_t dbase = 0;
  uint32_t dyn_static_pct = 35;  // QDC_DYN: static share of the fair share, % (100: off)
  // smallest granule (tiles per grab) of a reducing dynamic tail (QDC_DYN_GRAN, a power of two
  // <= 32): every granule writes its own partial per reduction slot, which k_dsum pre-sums —
  // C2's reverse passes at granule 2: ~43 000 partials per Gamma slot, ~0.35 GB per flush
  uint32_t dyn_gran_min = 1;
  // granule partials of dynamic-tail passes: [FIN_MAX][DYN_CAP][RED], slot i beside partials'
  cx* dparts = nullptr;
  cx* dsums = nullptr;  // [FIN_MAX][DYN_CAP / BLOCK][RED]: k_dsum's chunk sums
  static constexpr uint32_t DYN_CAP = 65536;  // 256 MiB of granule partials, allocated on first use
  std::vector<uint32_t> pending_nd;
  uint32_t last_ndyn = 0;  // granules of the last launch planned by plan_dyn (0: static)

  const char* init(int dev) {
    device = dev;
    QDC_HIP(hipSetDevice(dev));
    QDC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    QDC_HIP(hipMalloc(&partials, sizeof(cx) * (size_t)FIN_MAX * NBMAX * RED));
    QDC_HIP(hipMalloc(&results, sizeof(cx) * (size_t)FIN_MAX * RED));
    QDC_HIP(hipHostMalloc(&host_results, sizeof(cx) * (size_t)FIN_MAX * RED));
    QDC_HIP(hipMalloc(&dctr, sizeof(unsigned long long) * 8 * FG_DCTR_STRIDE));
    QDC_TRY(dyn_reset());
    if (const char* e = getenv("QDC_DYN")) dyn_static_pct = (uint32_t)std::max(0, atoi(e));
    if (const char* e = getenv("QDC_DYN_GRAN")) {
      const int v = atoi(e);
      dyn_gran_min = (v >= 1 && v <= 32 && (v & (v - 1)) == 0) ? (uint32_t)v : 1u;
    }
    if (const char* e = getenv("QDC_EVENT_FENCE"))
      prof.flags = atoi(e) ? (unsigned)hipEventDefault : (unsigned)hipEventDisableSystemFence;
    if (const char* e = getenv("QDC_GRID_CAP")) grid_cap = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_RED_CAP")) red_cap = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_REV_RED")) rev_red_cap = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_DIRECT_IT")) direct_it = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_TILE_FAR")) tile_far = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_XCD_MAP")) xcd_map = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_TILE2_WIDE")) tile2_wide = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_TILE1_WIDE")) tile1_wide = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_LANE")) lane_ops = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_DIAG_RU")) diag_ru = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_DIAG_Q")) diag_q = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_DIAG_RED")) diag_red = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_TILE_PF")) tile_pf = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_LANE_BLK")) lane_blk = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_LANE_TILE_BITS")) lane_tile_bits = strtoull(e, nullptr, 0);
    if (const char* e = getenv("QDC_LANE_NOBLK_BITS")) lane_noblk_bits = strtoull(e, nullptr, 0);
    if (const char* e = getenv("QDC_LANE_U")) {
      unsigned u0 = 0, u1 = 0, u2 = 0;
      if (sscanf(e, "%u,%u,%u", &u0, &u1, &u2) == 3) {
        lane_u[0] = u0;
        lane_u[1] = u1;
        lane_u[2] = u2;
      }
    }
    if (grid_cap < 1) grid_cap = 1;
    if (red_cap < 1) red_cap = 1;
    if (red_cap > NBMAX) red_cap = NBMAX;
    rev_red_cap = std::max(1u, std::min(rev_red_cap, NBMAX));
    diag_red = std::max(1u, std::min(diag_red, NBMAX));
    return nullptr;
  }
  // make this context's device current (launches and allocations of a shard go to its device)
  const char* use() const {
    int cur = -1;
    QDC_HIP(hipGetDevice(&cur));
    if (cur != device) QDC_HIP(hipSetDevice(device));
    return nullptr;
  }
  // Dynamic-tail tile counters of the one-wave register-resident passes (fgeo::dctr): host
  // and device agree on their value at each launch's start (dbase); re-zeroed at the start of
  // every circuit call, so a failed launch can never leave them out of step for the next call.
  const char* dyn_reset() {
    if (!dctr) return nullptr;
    QDC_HIP(hipMemsetAsync(dctr, 0, sizeof(unsigned long long) * 8 * FG_DCTR_STRIDE, stream));
    dbase = 0;
    return nullptr;
  }
  // static shares + dynamic tail of a launch of `grid` one-wave blocks over g.ntiles tiles:
  // every block runs dyn_static_pct % of its fair share block-contiguously (g.tpb tiles), the
  // rest is handed out by the eight pool counters; the counters then advance by ndyn / 8
  // successful grabs + grid / 8 final empty ones each, alike, which dbase follows
  // (false: no dynamic tail for this launch, g unchanged)
  // (false: no dynamic tail for this launch, g unchanged).  Granules of dgran tiles keep the
  // granule partials of a reducing pass within DYN_CAP per slot.
  bool plan_dyn(fgeo& g, uint32_t grid) {
    last_ndyn = 0;
    if (!QDC_DYN_TAIL || !dctr || dyn_static_pct >= 100 || (grid & 7u) || (g.ntiles & 7u) || g.order == 1)
      return false;
    if (g.ngrad > 0 && !dparts) {  // first reducing dynamic pass of this context
      if (hipMalloc(&dparts, sizeof(cx) * (size_t)FIN_MAX * DYN_CAP * RED) != hipSuccess ||
          hipMalloc(&dsums, sizeof(cx) * (size_t)FIN_MAX * (DYN_CAP / BLOCK) * RED) != hipSuccess) {
        (void)hipGetLastError();
        if (dparts) (void)hipFree(dparts);
        dparts = nullptr;
        dyn_static_pct = 100;  // no room: static shares only from now on
        return false;
      }
    }
    uint64_t per = g.ntiles * dyn_static_pct / 100 / grid;
    uint64_t ndyn = g.ntiles - per * grid;  // a multiple of 8 (ntiles and grid are)
    uint32_t gran = g.ngrad > 0 ? dyn_gran_min : 1u;
    if (g.ngrad > 0)
      while (ndyn / gran > DYN_CAP || (ndyn % (8ull * gran)) != 0) {
        if (gran >= 64) return false;
        gran *= 2;
        // whole granules: move the remainder of ndyn back into the static shares
        const uint64_t rem = ndyn % (8ull * gran);
        if (rem) {
          const uint64_t add = (rem + grid - 1) / grid;  // more static tiles per block
          per += add;
          if (per * grid > g.ntiles) return false;
          ndyn = g.ntiles - per * grid;
          gran = dyn_gran_min;  // re-check from the smallest granule with the new split
        }
      }
    if (ndyn == 0) return false;
    g.tpb = (uint32_t)per;
    g.nstat = per * grid;
    g.ndyn = ndyn;
    g.dgran = gran;
    g.dctr = dctr;
    g.dbase = dbase;
    g.dpart = dparts + pending_dst.size() * (size_t)DYN_CAP * RED;
    g.dstride = (uint64_t)DYN_CAP * RED;
    dbase += ndyn / gran / 8 + grid / 8;
    last_ndyn = g.ngrad > 0 ? (uint32_t)(ndyn / gran) : 0u;
    return true;
  }
  const char* sync() const {
    if (!stream) return nullptr;
    QDC_TRY(use());
    QDC_HIP(hipStreamSynchronize(stream));
    return nullptr;
  }
  void destroy() {
    DeviceGuard keep;
    if (stream) {
      (void)hipSetDevice(device);
      (void)hipStreamSynchronize(stream);
    }
    if (partials) (void)hipFree(partials);
    if (results) (void)hipFree(results);
    if (host_results) (void)hipHostFree(host_results);
    if (dctr) (void)hipFree(dctr);
    dctr = nullptr;
    if (dparts) (void)hipFree(dparts);
    if (dsums) (void)hipFree(dsums);
    dparts = dsums = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    partials = results = host_results = nullptr;
    stream = nullptr;
  }


  template <typename K, typename... Args>
  const char* launch(const char* name, double bytes, K kernel, uint32_t grid, Args... args) {
    return launch_block(name, bytes, kernel, grid, (uint32_t)BLOCK, args...);
  }
  template <typename K, typename... Args>
  const char* launch_block(const char* name, double bytes, K kernel, uint32_t grid,
                           uint32_t block, Args... args) {
    hipEvent_t a = nullptr, b = nullptr;
    if (prof.on) {
      a = prof.get();
      b = prof.get();
      if (a) (void)hipEventRecord(a, stream);
    }
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, stream, args...);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      return fail("HIP ERROR: launch of kernel %s failed with %s.", name, hipGetErrorName(e));
    if (prof.on && a && b) {
      (void)hipEventRecord(b, stream);
      prof.recs.push_back({name, bytes, next_flops, a, b});
    }
    next_flops = 0;
    return nullptr;
  }

  // launches of specialized kernels in this process (qdc_jit_stats: tests check that a forced
  // specialized run launched them, not the interpreted kernels)
  static std::atomic<uint64_t>& spec_launches() {
    static std::atomic<uint64_t> n{0};
    return n;
  }
  // a kernel from a loaded code object (qdc_jit.hpp), arguments as for launch_block
  template <typename... Args>
  const char* launch_module(const char* name, double bytes, hipFunction_t fn, uint32_t grid,
                            uint32_t block, Args... args) {
    hipEvent_t a = nullptr, b = nullptr;
    if (prof.on) {
      a = prof.get();
      b = prof.get();
      if (a) (void)hipEventRecord(a, stream);
    }
    void* params[] = {(void*)&args...};
    hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, stream, params, nullptr);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess)
      return fail("HIP ERROR: launch of kernel %s (specialized) failed with %s.", name,
                  hipGetErrorName(e));
    spec_launches().fetch_add(1, std::memory_order_relaxed);
    if (prof.on && a && b) {
      (void)hipEventRecord(b, stream);
      prof.recs.push_back({name, bytes, next_flops, a, b});
    }
    next_flops = 0;
    return nullptr;
  }

  // --- reduction slots -----------------------------------------------------------------
  // A reduction kernel writes its per-block partials into the next free slot; the slot is
  // later summed into base[dst*RED .. +RED) by k_finalize.  Pending slots may have different
  // bases (the local shards of a circuit each reduce into their own buffers: one flush per
  // shard launch was 8 finalize launches per pass at 8 shards, profiles/r5/r5c), not different
  // accumulate modes.
  const char* begin_reduction(cx* base, int accumulate) {
    if (accumulate != pending_accumulate) QDC_TRY(flush());
    pending_base = base;
    pending_accumulate = accumulate;
    if (pending_dst.size() == (size_t)FIN_MAX) QDC_TRY(flush());
    return nullptr;
  }
  cx* slot_ptr() const { return partials + pending_dst.size() * (size_t)NBMAX * RED; }
  // nd: granule partials of a dynamic-tail pass in the slot's dparts row (0: none)
  void commit(uint32_t dst, uint32_t nb, uint32_t nd = 0) {
    pending_dst.push_back(pending_base + (size_t)dst * RED);
    pending_nb.push_back(nb);
    pending_nd.push_back(nd);
  }
  const char* flush() {
    size_t i = 0;
    while (i < pending_dst.size()) {
      // group consecutive slots with equal partial counts into one launch
      size_t j = i;
      fin_table tab{};
      while (j < pending_dst.size() && pending_nb[j] == pending_nb[i] &&
             pending_nd[j] == pending_nd[i]) {
        tab.dst[j - i] = pending_dst[j];
        ++j;
      }
      const cx* p2 = dparts + i * (size_t)DYN_CAP * RED;
      uint64_t s2 = (uint64_t)DYN_CAP * RED;
      uint32_t n2 = pending_nd[i];
      if (n2 > (uint32_t)BLOCK) {  // many granules: pre-sum them in chunks of BLOCK (fixed order)
        const uint32_t nch = (n2 + BLOCK - 1) / BLOCK;
        const uint64_t os = (uint64_t)(DYN_CAP / BLOCK) * RED;
        cx* out = dsums + i * (size_t)(DYN_CAP / BLOCK) * RED;
        hipLaunchKernelGGL(k_dsum, dim3(nch, (uint32_t)(j - i)), dim3(BLOCK), 0, stream, p2, s2,
                           n2, out, os);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail("HIP ERROR: launch of kernel dsum failed with %s.", hipGetErrorName(e));
        p2 = out;
        s2 = os;
        n2 = nch;
      }
      QDC_TRY(launch("finalize", 0.0, k_finalize,
                     (uint32_t)(j - i), (const cx*)(partials + i * (size_t)NBMAX * RED),
                     (uint64_t)NBMAX * RED, pending_nb[i], tab, pending_accumulate, p2, s2,
                     n2));
      i = j;
    }
    pending_dst.clear();
    pending_nb.clear();
    pending_nd.clear();
    return nullptr;
  }
};

// ---------------------------------------------------------------------------------------
// Launch geometry (SURVEY.md §2.1 index rules, in 16-byte-chunk space)
// ---------------------------------------------------------------------------------------
struct Plan {
  bool tile = false;  // TILE family (a target at chunk bit 0..5) or DIRECT family
  bool lane = false;  // LANE family (overrides both; k_lane)
  int R = 2;
  int mode = 0;       // DIRECT row layout (see rows<R, MODE>)
  int ampk = -1;      // LANE: the gate bit held inside the chunk (f32 qubit 0), -1 none
  int lu = 1;         // LANE: units in flight per wave (1, 4 or 8)
  bool blk = false;   // LANE: the block-wide variant (k_lane_blk)
  geo g{};
  tgeo tg{};
  lgeo lg{};
};

inline uint64_t nchunks_of(uint32_t n) { return ((uint64_t)1 << n) / VEC; }
inline uint32_t log2u(uint64_t x) {
  uint32_t r = 0;
  while ((x >> r) > 1) ++r;
  return r;
}
// a target whose pair mate sits in another lane of the same wave
inline bool is_low(uint32_t q) { return q >= (uint32_t)LV && (q - LV) < (uint32_t)LOWBITS; }

// items per thread for block-contiguous iteration: keep the grid near `target` blocks
inline uint32_t per_thread(uint64_t items, uint32_t target) {
  uint64_t it = 1;
  while ((uint64_t)BLOCK * it * target < items) it <<= 1;
  return (uint32_t)it;
}

// q1: R = 2, pos2 == pos1 == target.  q2: R = 4.
inline Plan plan_gate(uint32_t n, int R, uint32_t pos2, uint32_t pos1, bool two_states,
                      uint32_t grid_target, bool far_tile = false, uint32_t wide2 = 0,
                      uint32_t wide1 = 0) {
  Plan p;
  p.R = R;
  const uint64_t nch = nchunks_of(n);
  const bool low = is_low(pos1) || (R == 4 && is_low(pos2));
  if (!low && !far_tile) {
    if (R == 2) {
      if ((int)pos1 < LV) {
        p.mode = 1;
        p.g.items = nch;
      } else {
        p.mode = 0;
        p.g.lo = pos1 - LV;
        p.g.sa = (uint64_t)1 << p.g.lo;
        p.g.items = nch / 2;
      }
    } else {
      const uint32_t lo = pos2 < pos1 ? pos2 : pos1;
      const uint32_t hi = pos2 < pos1 ? pos1 : pos2;
      if ((int)lo < LV) {
        p.mode = (lo == pos1) ? 1 : 2;
        p.g.hi = hi - LV;
        p.g.sa = (uint64_t)1 << p.g.hi;
        p.g.items = nch / 2;
      } else {
        p.mode = 0;
        p.g.lo = lo - LV;
        p.g.hi = hi - LV;
        p.g.sa = (uint64_t)1 << (pos2 - LV);
        p.g.sb = (uint64_t)1 << (pos1 - LV);
        p.g.items = nch / 4;
      }
    }
    p.g.it = per_thread(p.g.items, grid_target);
    return p;
  }
  // TILE: 256*K chunks per state per tile, K = 4 (one state) or 2 (two states)
  p.tile = true;
  // wide2: two-state tiles of 2^(9 + wide2) chunks; wide1: one-state tiles of 2^(10 + wide1)
  // (wide = 2: 64 KiB of LDS per block)
  const uint32_t T = two_states ? 9 + (wide2 > 2 ? 2 : wide2) : 10 + (wide1 > 2 ? 2 : wide1);
  const uint32_t cbits = log2u(nch);
  const uint32_t teff = cbits < T ? cbits : T;
  // targets at chunk bits beyond the tile's contiguous bits become row bits (each row bit
  // takes one contiguous bit, which may push a second target out: iterate)
  const uint32_t tq[2] = {pos1, pos2};
  const int nt = (R == 2) ? 1 : 2;
  uint32_t l = teff, h = 0, hb[2] = {0, 0};
  for (;;) {
    uint32_t k = 0, fb[2] = {0, 0};
    for (int i = 0; i < nt; ++i)
      if (tq[i] >= (uint32_t)LV && tq[i] - LV >= teff - h) fb[k++] = tq[i] - LV;
    if (k <= h) break;
    h = k;
    hb[0] = fb[0] < fb[1] || k == 1 ? fb[0] : fb[1];
    hb[1] = k == 1 ? 0 : (fb[0] < fb[1] ? fb[1] : fb[0]);
  }
  l = teff - h;
  const uint32_t hb0 = hb[0];
  auto local_bit = [&](uint32_t q) -> uint32_t {
    if (q < (uint32_t)LV || q - LV < l) return q;
    return (q - LV == hb0) ? LV + l : LV + l + 1;  // row bit 0 / 1
  };
  p.tg.l = l;
  p.tg.h = h;
  p.tg.hb0 = hb0;
  p.tg.hb1 = hb[1];
  p.tg.t1 = local_bit(pos1);
  p.tg.t2 = local_bit(pos2);
  p.tg.ntiles = nch >> (l + h);
  uint64_t tpb = 1;
  while (tpb * grid_target < p.tg.ntiles) tpb <<= 1;
  p.tg.tpb = (uint32_t)tpb;
  return p;
}

// LANE family geometry (k_lane): false when the state has fewer than 64 chunks.  Gate bit k
// (0: pos1 / the q1 target, 1: pos2) is the in-chunk bit (f32 qubit 0) or a lane bit: chunk
// bits below 6 - #far keep their own lane bit, the far ones take the top lane bits.
// ub = 10: the block-wide variant (k_lane_blk, 1024-chunk units, partners through LDS).
inline bool plan_lane(uint32_t n, int R, uint32_t pos2, uint32_t pos1, uint32_t grid_target,
                      bool reduces, Plan& p, uint32_t lu = 1, uint32_t ub = 6) {
  const uint64_t nch = nchunks_of(n);
  if (nch < ((uint64_t)1 << ub)) return false;
  const uint32_t pos[2] = {pos1, pos2};
  const int nt = (R == 2) ? 1 : 2;
  int ampk = -1;
  uint32_t t[2] = {0, 0};
  bool in_lane[2] = {false, false};
  for (int k = 0; k < nt; ++k) {
    if ((int)pos[k] < LV) {
      ampk = k;
    } else {
      t[k] = pos[k] - LV;
      in_lane[k] = true;
    }
  }
  uint32_t nf = 0;
  for (;;) {
    uint32_t cnt = 0;
    for (int k = 0; k < nt; ++k) cnt += (in_lane[k] && t[k] >= ub - nf) ? 1u : 0u;
    if (cnt <= nf) break;
    nf = cnt;
  }
  const uint32_t nlow = ub - nf;
  uint32_t far[2] = {0, 0}, nfar = 0;
  for (int k = 0; k < nt; ++k)
    if (in_lane[k] && t[k] >= nlow) far[nfar++] = t[k];
  if (nfar == 2 && far[0] > far[1]) std::swap(far[0], far[1]);
  auto lane_bit = [&](uint32_t c) -> uint32_t {
    if (c < nlow) return c;
    return nlow + ((nfar == 2 && c == far[1]) ? 1u : 0u);
  };
  p = Plan{};
  p.lane = true;
  p.R = R;
  p.ampk = ampk;
  lgeo& g = p.lg;
  g.units = nch >> ub;
  p.blk = ub > 6;
  g.nlow = nlow;
  g.nf = nfar;
  g.f0 = far[0];
  g.f1 = far[1];
  g.m0 = in_lane[0] ? (1u << lane_bit(t[0])) : 0u;
  g.m1 = (nt == 2 && in_lane[1]) ? (1u << lane_bit(t[1])) : 0u;
  // streaming: one step of lu units per wave; reductions: about grid_target blocks of 4 waves
  p.lu = (lu >= 8) ? 8 : (lu >= 4) ? 4 : 1;
  uint64_t it = (uint64_t)p.lu;
  if (reduces)
    while ((uint64_t)(BLOCK / 64) * it * grid_target < g.units) it <<= 1;
  g.it = (uint32_t)it;
  return true;
}

// ---------------------------------------------------------------------------------------
// Host small-matrix algebra (gates are 2x2 / 4x4, row-major).
// ---------------------------------------------------------------------------------------
template <int R>
inline mat<R> to_mat(const qdc_complex* h) {
  mat<R> m;
  for (int i = 0; i < R * R; ++i) m.a[i] = {h[i].re, h[i].im};
  return m;
}
template <int R>
inline mat<R> transpose(const mat<R>& m) {
  mat<R> t;
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < R; ++j) t.a[i * R + j] = m.a[j * R + i];
  return t;
}
template <int R>
inline mat<R> conj_transpose(const mat<R>& m) {
  mat<R> t;
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < R; ++j) t.a[i * R + j] = {m.a[j * R + i].x, -m.a[j * R + i].y};
  return t;
}
inline diag4 to_diag(const qdc_complex* h) {
  diag4 d;
  for (int i = 0; i < 4; ++i) d.a[i] = {h[i].re, h[i].im};
  return d;
}
inline diag4 conj_diag(const diag4& d) {
  diag4 c;
  for (int i = 0; i < 4; ++i) c.a[i] = {d.a[i].x, -d.a[i].y};
  return c;
}

// Inverse of a row-major R x R matrix, restating cublas{C,Z}matinvBatched as the reference
// calls it (primitives.cu:114-138): cuBLAS is column-major, so it factorises A^T by LU with
// partial pivoting; info = i (1-based) when U(i,i) is exactly zero → "U(i, i) is zero.".
// Computed in long double, rounded once to the working precision.
template <int R>
inline const char* inverse(const mat<R>& a, mat<R>& out) {
  using C = std::complex<long double>;
  C m[R][R], inv[R][R];
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < R; ++j) {
      // column-major view of the row-major buffer: M = A^T
      m[i][j] = C(a.a[j * R + i].x, a.a[j * R + i].y);
      inv[i][j] = (i == j) ? C(1, 0) : C(0, 0);
    }
  for (int k = 0; k < R; ++k) {
    int piv = k;
    long double best = std::abs(m[k][k]);
    for (int r = k + 1; r < R; ++r) {
      long double v = std::abs(m[r][k]);
      if (v > best) {
        best = v;
        piv = r;
      }
    }
    if (best == 0.0L) return fail("U(%d, %d) is zero.", k + 1, k + 1);
    if (piv != k)
      for (int j = 0; j < R; ++j) {
        std::swap(m[k][j], m[piv][j]);
        std::swap(inv[k][j], inv[piv][j]);
      }
    const C d = m[k][k];
    for (int j = 0; j < R; ++j) {
      m[k][j] /= d;
      inv[k][j] /= d;
    }
    for (int r = 0; r < R; ++r) {
      if (r == k) continue;
      const C f = m[r][k];
      if (f == C(0, 0)) continue;
      for (int j = 0; j < R; ++j) {
        m[r][j] -= f * m[k][j];
        inv[r][j] -= f * inv[k][j];
      }
    }
  }
  // inv = (A^T)^-1 = (A^-1)^T; its column-major storage is A^-1 row-major.
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < R; ++j)
      out.a[i * R + j] = {(real)inv[j][i].real(), (real)inv[j][i].imag()};
  return nullptr;
}

// ---------------------------------------------------------------------------------------
// Op launchers (all asynchronous on ctx.stream)
// ---------------------------------------------------------------------------------------
inline double state_bytes(uint32_t n) { return (double)((uint64_t)1 << n) * sizeof(cx); }

// items in flight per thread and step of the direct family: 4 q1 items (8 chunks per state),
// 2 q2 items
constexpr int direct_u(int R) { return R == 2 ? 4 : 2; }

inline uint32_t blocks_of(const Plan& p) {
  if (p.lane && p.blk) return (uint32_t)p.lg.units;
  if (p.lane) {
    const uint64_t per = (uint64_t)(BLOCK / 64) * p.lg.it;
    return (uint32_t)((p.lg.units + per - 1) / per);
  }
  if (p.tile) return (uint32_t)((p.tg.ntiles + p.tg.tpb - 1) / p.tg.tpb);
  return (uint32_t)((p.g.items + (uint64_t)BLOCK * p.g.it - 1) / ((uint64_t)BLOCK * p.g.it));
}

template <int OP, int R, int U>
inline const char* run_lane(Ctx& c, const char* name, double bytes, chunk* fc, chunk* bc,
                            const mat<R>& A, const mat<R>& B, const Plan& p, uint32_t grid,
                            cx* partials) {
  if (p.ampk < 0)
    return c.launch(name, bytes, k_lane<OP, R, -1, U>, grid, fc, bc, A, B, p.lg, partials);
  if constexpr (VEC == 2) {
    if (p.ampk == 0)
      return c.launch(name, bytes, k_lane<OP, R, 0, U>, grid, fc, bc, A, B, p.lg, partials);
    if constexpr (R == 4)
      return c.launch(name, bytes, k_lane<OP, 4, 1, U>, grid, fc, bc, A, B, p.lg, partials);
  }
  return fail("invalid lane plan");
}

// Launch one gate-shaped op (any OP, R) on the family the plan selected.
template <int OP, int R>
inline const char* run_op(Ctx& c, const char* name, double bytes, cx* f, cx* b, const mat<R>& A,
                          const mat<R>& B, const Plan& p, cx* partials) {
  chunk* fc = reinterpret_cast<chunk*>(f);
  chunk* bc = reinterpret_cast<chunk*>(b);
  const uint32_t grid = blocks_of(p);
  if (p.lane && p.blk) {
    if constexpr (OP == OP_APPLY || OP == OP_INJECT || OP == OP_INJECT_FIRST) {
      // 1024-thread blocks (one unit each)
      if (p.ampk < 0)
        return c.launch_block(name, bytes, k_lane_blk<OP, R, -1>, grid, (uint32_t)LB_NT, fc, bc, A, p.lg);
      if constexpr (VEC == 2) {
        if (p.ampk == 0)
          return c.launch_block(name, bytes, k_lane_blk<OP, R, 0>, grid, (uint32_t)LB_NT, fc, bc, A, p.lg);
        if constexpr (R == 4)
          return c.launch_block(name, bytes, k_lane_blk<OP, 4, 1>, grid, (uint32_t)LB_NT, fc, bc, A, p.lg);
      }
    }
    return fail("invalid block lane plan");
  }
  if (p.lane) {
    if (p.lu == 8) return run_lane<OP, R, 8>(c, name, bytes, fc, bc, A, B, p, grid, partials);
    if (p.lu == 4) return run_lane<OP, R, 4>(c, name, bytes, fc, bc, A, B, p, grid, partials);
    return run_lane<OP, R, 1>(c, name, bytes, fc, bc, A, B, p, grid, partials);
  }
  if (p.tile) {
    constexpr int K = op_two_states(OP) ? 2 : 4;
    if (K == 2 && p.tg.l + p.tg.h > 10)  // the widest two-state tile (QDC_TILE2_WIDE=2)
      return c.launch(name, bytes, k_tile<OP, R, 8>, grid, fc, bc, A, B, p.tg, partials);
    if (K == 2 && p.tg.l + p.tg.h > 9)  // a wide two-state tile (QDC_TILE2_WIDE)
      return c.launch(name, bytes, k_tile<OP, R, 4>, grid, fc, bc, A, B, p.tg, partials);
    if (K == 4 && p.tg.l + p.tg.h > 11)  // the widest one-state tile (QDC_TILE1_WIDE=2)
      return c.launch(name, bytes, k_tile<OP, R, 16>, grid, fc, bc, A, B, p.tg, partials);
    if (K == 4 && p.tg.l + p.tg.h > 10)  // a wide one-state tile (QDC_TILE1_WIDE)
      return c.launch(name, bytes, k_tile<OP, R, 8>, grid, fc, bc, A, B, p.tg, partials);
    return c.launch(name, bytes, k_tile<OP, R, K>, grid, fc, bc, A, B, p.tg, partials);
  }
  if (p.mode == 0)
    return c.launch(name, bytes, k_direct<OP, R, 0, direct_u(R)>, grid, fc, bc, A, B, p.g,
                    partials);
  if (p.mode == 1)
    return c.launch(name, bytes, k_direct<OP, R, 1, direct_u(R)>, grid, fc, bc, A, B, p.g,
                    partials);
  if constexpr (R == 4)
    return c.launch(name, bytes, k_direct<OP, 4, 2, direct_u(4)>, grid, fc, bc, A, B, p.g, partials);
  return fail("invalid plan");
}

template <int R>
inline Plan plan_for(const Ctx& c, uint32_t n, uint32_t pos2, uint32_t pos1, bool two,
                     bool reduces, bool writes_both = false) {
  const uint32_t cls = writes_both ? 0u : two ? 2u : 1u;  // QDC_TILE_FAR bit
  Plan p;
  const uint32_t lcls = writes_both ? 0u : reduces ? 2u : 1u;  // QDC_LANE bit
  const uint32_t rcap = writes_both ? c.rev_red_cap : c.red_cap;
  // byte-stride bits of the targets (Ctx::lane_tile_bits / lane_noblk_bits)
  constexpr uint32_t CXB = sizeof(cx) == 8 ? 3u : 4u;
  const uint64_t tb = ((uint64_t)1 << (pos1 + CXB)) | ((uint64_t)1 << (pos2 + CXB));
  const bool apply1 = lcls == 1 && !two;  // a one-state application (not an injection)
  const bool lane_tile = apply1 && R == 2 && (tb & c.lane_tile_bits) != 0;
  if (!((c.lane_ops >> lcls) & 1u) || lane_tile ||
      !plan_lane(n, R, pos2, pos1, rcap, reduces, p, c.lane_u[lcls])) {
    p = plan_gate(n, R, pos2, pos1, two, reduces ? rcap : c.grid_cap,
                  (c.tile_far >> cls) & 1u, c.tile2_wide, c.tile1_wide);
    if (!p.tile && p.g.it < c.direct_it) p.g.it = c.direct_it;
  } else if (lcls == 1 && c.lane_blk && p.lg.nf > 0 && !(apply1 && (tb & c.lane_noblk_bits))) {
    // a far target: the block-wide variant, when the state holds a 1024-chunk unit
    Plan q;
    if (plan_lane(n, R, pos2, pos1, c.red_cap, reduces, q, 1, 10)) p = q;
  }
  // XCD-aware order for streaming launches only by default: reductions (few long-lived blocks
  // with contiguous ranges) measured slower with it (density 85 -> 73-82 %, profiles/r2s_*)
  p.g.xcd = p.tg.xcd = p.lg.xcd = (c.xcd_map >> (reduces ? 1 : 0)) & 1u;  // bit 0 streaming, 1 reducing
  // except two-state tiles whose two row bits both sit at chunk bit >= 20 (q2 pairs of far
  // qubits, row strides >= 16 MiB): XCD order measured better there, reverse_q2 (26,27)
  // 74.0 -> 75.6 %, while (14,13) drops 73.3 -> 69.1 and (5,20) / (27,0) lose 3-4 points
  // (profiles/r6/r6o)
  if (p.tile && two && reduces && p.tg.h == 2 && p.tg.hb0 >= 20) p.tg.xcd = 1;
  p.g.gm = c.gm;
  p.tg.gm = c.gm;
  p.tg.pf = c.tile_pf && p.tg.h == 0;
  p.lg.gm = c.gm;
  return p;
}

template <int R>
inline const char* apply_dense(Ctx& c, cx* s, const mat<R>& m, uint32_t pos2, uint32_t pos1,
                               uint32_t n, const char* name) {
  const Plan p = plan_for<R>(c, n, pos2, pos1, false, false);
  return run_op<OP_APPLY, R>(c, name, 2.0 * state_bytes(n), s, nullptr, m, m, p, nullptr);
}

inline dgeo diag_geo(const Ctx& c, uint32_t n, uint32_t pos2, uint32_t pos1, uint32_t target) {
  dgeo g;
  g.gm = c.gm;
  g.nchunks = nchunks_of(n);
  g.it = per_thread(g.nchunks, target);
  if (target == c.grid_cap && g.it < c.direct_it) g.it = c.direct_it;  // streaming
  g.p2 = pos2;
  g.p1 = pos1;
  g.xcd = (c.xcd_map >> 2) & 1u;  // QDC_XCD_MAP bit 2: diagonal launches
  return g;
}
inline uint32_t diag_blocks(const dgeo& g) {
  return (uint32_t)((g.nchunks + (uint64_t)BLOCK * g.it - 1) / ((uint64_t)BLOCK * g.it));
}
// k_diag_q's geometry (qdc_kernels.hpp): false when the state does not split into whole
// blocks of one quadrant each (small states), or when it is not a multiple of the kernel's U
// chunks in flight — k_diag runs those
inline bool diag_q_geo(const dgeo& g, dqgeo& q, uint32_t U) {
  if (g.nchunks == 0 || (g.nchunks & (g.nchunks - 1)) != 0 || g.it % U != 0) return false;
  uint32_t lognc = 0;
  while (((uint64_t)1 << lognc) < g.nchunks) ++lognc;
  q = dqgeo{};
  q.gm = g.gm;
  q.it = g.it;
  uint32_t cb[2], nb = 0;
  auto enc = [&](uint32_t p) -> uint32_t {
    if (p < (uint32_t)LV) return 0x100u;
    const uint32_t c = p - (uint32_t)LV;
    if (c < 8) return 0x200u | c;
    cb[nb++] = c;
    return 0x400u | c;  // quadrant bit resolved below
  };
  q.k1 = enc(g.p1);
  q.k2 = enc(g.p2);
  if (nb == 2 && cb[0] > cb[1]) std::swap(cb[0], cb[1]);
  for (uint32_t* k : {&q.k1, &q.k2})
    if (*k & 0x400u) *k = 0x400u | ((*k & 0xffu) == cb[0] ? 0u : 1u);
  q.nb = nb;
  q.c0 = nb >= 1 ? cb[0] : 0;
  q.c1 = nb >= 2 ? cb[1] : 0;
  if (lognc < nb) return false;
  q.qshift = lognc - nb;
  const uint64_t span = (uint64_t)BLOCK * g.it;  // chunks per block
  return span <= ((uint64_t)1 << q.qshift) && g.nchunks % span == 0;
}

inline const char* apply_diag(Ctx& c, cx* s, const diag4& d, uint32_t pos2, uint32_t pos1,
                              uint32_t n, const char* name) {
  const dgeo g = diag_geo(c, n, pos2, pos1, c.grid_cap);
  return c.launch(name, 2.0 * state_bytes(n), k_diag<DIAG_APPLY, 4>, diag_blocks(g),
                  reinterpret_cast<chunk*>(s), (chunk*)nullptr, d, d, g, (cx*)nullptr);
}

// reduction slot helper: run `launch(partials)` producing `nb` partials for base[dst]
template <class F>
inline const char* reduce_into(Ctx& c, cx* base, uint32_t dst, int accumulate, uint32_t nb,
                               F&& launch) {
  if (nb > NBMAX) return fail("reduction grid %u exceeds %u", nb, NBMAX);
  QDC_TRY(c.begin_reduction(base, accumulate));
  QDC_TRY(launch(c.slot_ptr()));
  c.commit(dst, nb);
  return nullptr;
}

// density of one (R = 2) or two (R = 4) qubits → reduction slot for base[dst]
template <int R>
inline const char* density(Ctx& c, const cx* s, uint32_t pos2, uint32_t pos1, uint32_t n,
                           cx* base, uint32_t dst, int accumulate) {
  const Plan p = plan_for<R>(c, n, pos2, pos1, false, true);
  const mat<R> z{};
  return reduce_into(c, base, dst, accumulate, blocks_of(p), [&](cx* out) {
    return run_op<OP_DENSITY, R>(c, R == 2 ? "density_q1" : "density_q2", state_bytes(n),
                                 const_cast<cx*>(s), nullptr, z, z, p, out);
  });
}

template <int R>
inline const char* grad_dense(Ctx& c, const cx* f, const cx* b, uint32_t pos2, uint32_t pos1,
                              uint32_t n, cx* base, uint32_t dst, int accumulate) {
  const Plan p = plan_for<R>(c, n, pos2, pos1, true, true);
  const mat<R> z{};
  return reduce_into(c, base, dst, accumulate, blocks_of(p), [&](cx* out) {
    return run_op<OP_GRAD, R>(c, R == 2 ? "grad_q1" : "grad_q2", 2.0 * state_bytes(n),
                              const_cast<cx*>(f), const_cast<cx*>(b), z, z, p, out);
  });
}

inline const char* grad_diag(Ctx& c, const cx* f, const cx* b, uint32_t pos2, uint32_t pos1,
                             uint32_t n, cx* base, uint32_t dst, int accumulate) {
  const dgeo g = diag_geo(c, n, pos2, pos1, c.red_cap);
  const diag4 z{};
  return reduce_into(c, base, dst, accumulate, diag_blocks(g), [&](cx* out) {
    return c.launch("grad_q2_diag", 2.0 * state_bytes(n), k_diag<DIAG_GRAD, 4>, diag_blocks(g),
                    const_cast<chunk*>(reinterpret_cast<const chunk*>(f)),
                    const_cast<chunk*>(reinterpret_cast<const chunk*>(b)), z, z, g, out);
  });
}

// Fused reverse step for a dense gate.  grad_base == nullptr → constant gate (no gradient).
template <int R>
inline const char* reverse_dense(Ctx& c, cx* f, cx* b, const mat<R>& A, const mat<R>& B,
                                 uint32_t pos2, uint32_t pos1, uint32_t n, cx* grad_base,
                                 uint32_t dst) {
  const double bytes = 4.0 * state_bytes(n);
  const char* name = (R == 2) ? "reverse_q1" : "reverse_q2";
  if (grad_base) {
    const Plan p = plan_for<R>(c, n, pos2, pos1, true, true, true);
    return reduce_into(c, grad_base, dst, 0, blocks_of(p), [&](cx* out) {
      return run_op<OP_REVERSE_GRAD, R>(c, name, bytes, f, b, A, B, p, out);
    });
  }
  const Plan p = plan_for<R>(c, n, pos2, pos1, true, false, true);
  return run_op<OP_REVERSE, R>(c, name, bytes, f, b, A, B, p, nullptr);
}

inline const char* reverse_diag(Ctx& c, cx* f, cx* b, const diag4& d, uint32_t pos2,
                                uint32_t pos1, uint32_t n, cx* grad_base, uint32_t dst) {
  chunk* fc = reinterpret_cast<chunk*>(f);
  chunk* bc = reinterpret_cast<chunk*>(b);
  const diag4 dc = conj_diag(d);
  const double bytes = 4.0 * state_bytes(n);
  if (c.diag_q) {  // k fixed per thread (k_diag_q), when the state splits into whole blocks
    const uint32_t U = c.diag_ru >= 16 ? 16u : c.diag_ru >= 8 ? 8u : 4u;
    dgeo g = diag_geo(c, n, pos2, pos1, grad_base ? c.diag_red : c.grid_cap);
    g.it = std::max(g.it, U);
    dqgeo q;
    if (diag_q_geo(g, q, U)) {
      const uint32_t nb = diag_blocks(g);
      auto go = [&](auto kern, cx* out) { return c.launch("reverse_q2_diag", bytes, kern, nb, fc, bc, dc, d, q, out); };
      if (grad_base)
        return reduce_into(c, grad_base, dst, 0, nb, [&](cx* out) {
          return U == 16 ? go(k_diag_q<DIAG_REVERSE_GRAD, 16>, out)
                 : U == 8 ? go(k_diag_q<DIAG_REVERSE_GRAD, 8>, out)
                          : go(k_diag_q<DIAG_REVERSE_GRAD, 4>, out);
        });
      return U == 16 ? go(k_diag_q<DIAG_REVERSE, 16>, nullptr)
             : U == 8 ? go(k_diag_q<DIAG_REVERSE, 8>, nullptr)
                      : go(k_diag_q<DIAG_REVERSE, 4>, nullptr);
    }
  }
  if (grad_base) {
    const dgeo g = diag_geo(c, n, pos2, pos1, c.red_cap);
    return reduce_into(c, grad_base, dst, 0, diag_blocks(g), [&](cx* out) {
      if (c.diag_ru >= 8)
        return c.launch("reverse_q2_diag", bytes, k_diag<DIAG_REVERSE_GRAD, 8>, diag_blocks(g),
                        fc, bc, dc, d, g, out);
      return c.launch("reverse_q2_diag", bytes, k_diag<DIAG_REVERSE_GRAD, 2>, diag_blocks(g), fc,
                      bc, dc, d, g, out);
    });
  }
  const dgeo g = diag_geo(c, n, pos2, pos1, c.grid_cap);
  if (c.diag_ru >= 8)
    return c.launch("reverse_q2_diag", bytes, k_diag<DIAG_REVERSE, 8>, diag_blocks(g), fc, bc,
                    dc, d, g, (cx*)nullptr);
  return c.launch("reverse_q2_diag", bytes, k_diag<DIAG_REVERSE, 2>, diag_blocks(g), fc, bc, dc,
                  d, g, (cx*)nullptr);
}

template <int R>
inline const char* inject(Ctx& c, const cx* f, cx* b, const mat<R>& m, uint32_t pos2,
                          uint32_t pos1, uint32_t n, bool first) {
  const Plan p = plan_for<R>(c, n, pos2, pos1, true, false);
  const double bytes = (first ? 2.0 : 3.0) * state_bytes(n);
  const char* name = (R == 2) ? "inject_q1" : "inject_q2";
  if (first)
    return run_op<OP_INJECT_FIRST, R>(c, name, bytes, const_cast<cx*>(f), b, m, m, p, nullptr);
  return run_op<OP_INJECT, R>(c, name, bytes, const_cast<cx*>(f), b, m, m, p, nullptr);
}

// op 0: dst = src; op 1: dst = 2 conj(src); op 2: dst += src; op 3: dst = |0..0>; op 4: 0.
// gm: dst is a state of an interleaved pair (Ctx::gm), src plain
template <int OP>
inline const char* elementwise(Ctx& c, const cx* src, cx* dst, uint32_t n, uint64_t gm = 0) {
  const uint64_t amps = (uint64_t)1 << n;
  const uint64_t nch = amps / VEC > 0 ? amps / VEC : 1;
  const uint32_t it = per_thread(nch, c.grid_cap);
  const uint32_t grid = (uint32_t)((nch + (uint64_t)BLOCK * it - 1) / ((uint64_t)BLOCK * it));
  const double bytes = (OP == 2 ? 3.0 : OP >= 3 ? 1.0 : 2.0) * state_bytes(n);
  static const char* names[5] = {"copy", "conj_and_double", "add", "set_standard", "zero"};
  return c.launch(names[OP], bytes, k_elementwise<OP>, grid, src, dst, amps, it, gm);
}

// the same kernels over an arbitrary number of complex values (reduction buffers)
template <int OP>
inline const char* elementwise_count(Ctx& c, const cx* src, cx* dst, uint64_t count) {
  const uint64_t nch = count / VEC > 0 ? count / VEC : 1;
  const uint32_t it = per_thread(nch, c.grid_cap);
  const uint32_t grid = (uint32_t)((nch + (uint64_t)BLOCK * it - 1) / ((uint64_t)BLOCK * it));
  return c.launch("reduce_sum", 0.0, k_elementwise<OP>, grid, src, dst, count, it, (uint64_t)0);
}

// remap pack of one shard of nl local qubits (victims: ascending amplitude positions >= 1);
// unpack: its inverse (victim blocks scattered back to the victim bits)
inline const char* pack(Ctx& c, const cx* src, cx* dst, const unsigned* victims, uint32_t g,
                        uint32_t nl, bool unpack = false) {
  packgeo pg{};
  pg.nchunks = nchunks_of(nl);
  pg.lowc = (nl - g) - LV;
  pg.g = g;
  for (uint32_t k = 0; k < g; ++k) pg.vc[k] = victims[k] - LV;
  // LDS tiles (k_pack_tile) whenever a tile fits the shard: every victim layout moves at
  // streaming rates (QDC_PACK_TILE=0: the direct kernel)
  static const bool tiled = [] {
    const char* e = getenv("QDC_PACK_TILE");
    return !(e && atoi(e) == 0);
  }();
  if (tiled && g <= 3 && pg.nchunks >= ((uint64_t)2 << PACK_KB) && pg.lowc >= PACK_KB) {
    packtile pt{};
    pt.nchunks = pg.nchunks;
    pt.lowc = pg.lowc;
    pt.g = g;
    for (uint32_t k = 0; k < g; ++k) {
      pt.vc[k] = pg.vc[k];
      pt.nv += pg.vc[k] < PACK_KB ? 1u : 0u;
    }
    const uint32_t tgrid = (uint32_t)(pg.nchunks >> PACK_KB);
    const char* cs = reinterpret_cast<const char*>(src);
    if (unpack)
      return c.launch("remap_unpack", 2.0 * state_bytes(nl), k_pack_tile<true>, tgrid,
                      reinterpret_cast<const chunk*>(cs), reinterpret_cast<chunk*>(dst), pt);
    return c.launch("remap_pack", 2.0 * state_bytes(nl), k_pack_tile<false>, tgrid,
                    reinterpret_cast<const chunk*>(cs), reinterpret_cast<chunk*>(dst), pt);
  }
  const uint32_t grid = (uint32_t)((pg.nchunks + BLOCK - 1) / BLOCK);
  if (unpack)
    return c.launch("remap_unpack", 2.0 * state_bytes(nl), k_pack<true>, grid,
                    reinterpret_cast<const chunk*>(src), reinterpret_cast<chunk*>(dst), pg);
  return c.launch("remap_pack", 2.0 * state_bytes(nl), k_pack<false>, grid,
                  reinterpret_cast<const chunk*>(src), reinterpret_cast<chunk*>(dst), pg);
}

// one run of diagonal cotangent injections (k_diag_inject): acc = false starts bwd
inline const char* diag_inject(Ctx& c, const cx* f, cx* b, const diag_tab& T, uint32_t ngroups,
                               uint32_t n, uint64_t gm, bool acc) {
  const uint64_t amps = (uint64_t)1 << n;
  const uint64_t nch = amps / VEC > 0 ? amps / VEC : 1;
  if (amps < (uint64_t)VEC) return fail("internal: diagonal injection on a state below one chunk");
  const uint32_t it = per_thread(nch, c.grid_cap);
  const uint32_t grid = (uint32_t)((nch + (uint64_t)BLOCK * it - 1) / ((uint64_t)BLOCK * it));
  const double bytes = (acc ? 3.0 : 2.0) * state_bytes(n);
  const chunk* fc = reinterpret_cast<const chunk*>(f);
  chunk* bc = reinterpret_cast<chunk*>(b);
  if (acc) return c.launch("inject_diag", bytes, k_diag_inject<true>, grid, fc, bc, T, nch, it, gm, ngroups);
  return c.launch("inject_diag", bytes, k_diag_inject<false>, grid, fc, bc, T, nch, it, gm, ngroups);
}

inline const char* set_standard(Ctx& c, cx* s, uint32_t n) {
  return elementwise<3>(c, nullptr, s, n);
}

}  // namespace qdc
