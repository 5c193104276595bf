// qdc_circuit.hpp — the circuit interpreter (src/circuit.rs:53-430 and the QuantizedTensor
// methods it calls, src/quantized_tensor.rs:54-238) as a native C++ runtime.
//
// Device state per circuit: `initial` (set_state_from_vector target), `state` (the forward
// state; the reverse sweep uncomputes it in place, exactly as circuit.rs:275 borrows
// self.state), `bwd` (the cotangent state, allocated on the first backward and kept), a
// gradient buffer and a density buffer.  That is 3 full states, never the reference's
// transient 4th (`conj_and_double` allocation per density injection, quantized_tensor.rs:81-86).
#pragma once

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include <rccl/rccl.h>

#include "qdc/circuit.h"
#include "qdc_device.hpp"
#include "qdc_shard.hpp"
#include "qdc_stage.hpp"
#include "qdc_fusion.hpp"
#include "qdc_jit.hpp"

namespace qdc {

// A flattened list of host buffers (gate matrices or density cotangents).
struct Flat {
  const qdc_complex* data;
  std::vector<size_t> off;
  std::vector<size_t> len;
  Flat(const qdc_complex* d, const size_t* lens, size_t n) : data(d), off(n), len(n) {
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
      off[i] = o;
      len[i] = lens[i];
      o += lens[i];
    }
  }
  size_t size() const { return len.size(); }
  const qdc_complex* at(size_t i) const { return data + off[i]; }
};

// The assertion sequence of QuantizedTensor::apply_* (quantized_tensor.rs:100-152).
inline const char* check_gate(const Instr& in, size_t len, uint32_t n) {
  if (len != (size_t)gate_len(in.kind)) return fail("Incorrect len of the gate's buffer.");
  if (is_q1_gate(in.kind)) {
    if (in.a >= n) return fail("pos is out of the bound.");
  } else {
    if (in.a == in.b) return fail("pos1 and pos2 must be different.");
    if (in.b >= n) return fail("pos1 is out of the bound.");
    if (in.a >= n) return fail("pos2 is out of the bound.");
  }
  return nullptr;
}
inline const char* check_density_pos(const Instr& in, uint32_t n) {
  if (is_q1_density(in.kind)) {
    if (in.a >= n) return fail("pos is out of the bound.");
  } else {
    if (in.a == in.b) return fail("pos1 and pos2 must be different.");
    if (in.b >= n) return fail("pos1 is out of the bound.");
    if (in.a >= n) return fail("pos2 is out of the bound.");
  }
  return nullptr;
}

#define QDC_NCCL(call)                                                                   \
  do {                                                                                   \
    ncclResult_t qdc_r_ = (call);                                                        \
    if (qdc_r_ != ncclSuccess)                                                           \
      return ::qdc::fail("RCCL ERROR: call of a function \"%s\" in line %d of file %s "  \
                         "failed with %s.",                                              \
                         #call, __LINE__, __FILE__, ncclGetErrorString(qdc_r_));          \
  } while (0)

// Per-device resources of a circuit: a context (stream, reduction arena, profiling) and the
// device copy of the fused-pass program.  One per shard when the shards run on their own
// streams (single-process multi-GPU, or the multi-stream rehearsal on one GPU), else one shared
// by every local shard.
struct DevRes {
  Ctx ctx;
  unsigned char* prog_dev = nullptr;
};

struct Shard {
  cx* initial = nullptr;
  cx* state = nullptr;
  cx* bwd = nullptr;
  bool bwd_live = false;  // bwd holds a cotangent (written by a backward): readable
  cx* scratch = nullptr;  // all-to-all staging (allocated when world > 1)
  std::vector<void*> owned;  // state allocations (remaps swap the pointers above among them)
  cx* dens = nullptr;
  cx* grads = nullptr;
  DevRes* d = nullptr;  // the shard's device resources
  Ctx& c() const { return d->ctx; }
};

// The shard exchange.  Transports:
//   * RCCL, one shard per process (one rank per GPU, xGMI): `comm`;
//   * RCCL, every shard of the job in this process, one per GPU (ncclCommInitAll): `comms`,
//     one collective per shard inside ncclGroupStart/End, each on its shard's stream;
//   * loopback, every shard on this process's one GPU: device-to-device copies — on one shared
//     stream, or (`multi_stream`) on the shards' own streams ordered by events.
struct Exchange {
  int world = 1;   // total shards
  int rank0 = 0;   // global index of this process's first shard
  int nlocal = 1;  // shards held by this process
  ncclComm_t comm = nullptr;
  std::vector<ncclComm_t> comms;
  bool multi_stream = false;
  std::vector<hipEvent_t> ev;  // multi_stream: one per shard

  static ncclDataType_t type() { return sizeof(real) == 4 ? ncclFloat : ncclDouble; }
  const char* events(size_t n) {
    while (ev.size() < n) {
      hipEvent_t e;
      QDC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ev.push_back(e);
    }
    return nullptr;
  }
  // every shard stream waits for every other shard stream's work so far
  const char* join(std::vector<Shard>& sh) {
    QDC_TRY(events(sh.size()));
    for (size_t s = 0; s < sh.size(); ++s) {
      QDC_TRY(sh[s].c().use());
      QDC_HIP(hipEventRecord(ev[s], sh[s].c().stream));
    }
    for (size_t d = 0; d < sh.size(); ++d)
      for (size_t s = 0; s < sh.size(); ++s)
        if (s != d) QDC_HIP(hipStreamWaitEvent(sh[d].c().stream, ev[s], 0));
    return nullptr;
  }
  void prof_begin(Shard& s, hipEvent_t& a, hipEvent_t& b) {
    Ctx& c = s.c();
    a = b = nullptr;
    if (c.prof.on) {
      a = c.prof.get();
      b = c.prof.get();
      if (a) (void)hipEventRecord(a, c.stream);
    }
  }
  void prof_end(Shard& s, hipEvent_t a, hipEvent_t b, double bytes) {
    Ctx& c = s.c();
    if (c.prof.on && a && b) {
      (void)hipEventRecord(b, c.stream);
      c.prof.recs.push_back({"alltoall", bytes, 0.0, a, b});  // link bytes, not HBM bytes
    }
  }

  // Block j of send[s] (chunk amplitudes) goes to shard j and lands as block s of recv[j].
  const char* alltoall(std::vector<Shard>& sh, std::vector<cx*>& send, std::vector<cx*>& recv,
                       size_t chunk) {
    if (world == 1) return nullptr;
    const double bytes = (double)chunk * sizeof(cx) * (world - 1);  // per shard
    std::vector<hipEvent_t> pa(sh.size()), pb(sh.size());
    for (size_t s = 0; s < sh.size(); ++s) prof_begin(sh[s], pa[s], pb[s]);
    if (comm) {
      QDC_NCCL(ncclAllToAll(send[0], recv[0], chunk * 2, type(), comm, sh[0].c().stream));
    } else if (!comms.empty()) {
      QDC_NCCL(ncclGroupStart());
      for (size_t s = 0; s < sh.size(); ++s)
        QDC_NCCL(ncclAllToAll(send[s], recv[s], chunk * 2, type(), comms[s], sh[s].c().stream));
      QDC_NCCL(ncclGroupEnd());
    } else {
      if (multi_stream) QDC_TRY(join(sh));  // sources written, destinations free
      for (int d = 0; d < nlocal; ++d)
        for (int s = 0; s < nlocal; ++s)
          QDC_HIP(hipMemcpyAsync(recv[d] + (size_t)s * chunk, send[s] + (size_t)d * chunk,
                                 chunk * sizeof(cx), hipMemcpyDeviceToDevice, sh[d].c().stream));
      if (multi_stream) QDC_TRY(join(sh));  // no source is rewritten before every copy is done
    }
    for (size_t s = 0; s < sh.size(); ++s) prof_end(sh[s], pa[s], pb[s], bytes);
    return nullptr;
  }
  // in-place sum over all shards of `count` complex values (every shard's buffer holds the sum)
  const char* allreduce(std::vector<Shard>& sh, std::vector<cx*>& bufs, size_t count) {
    if (world == 1 || count == 0) return nullptr;
    if (comm) {
      QDC_NCCL(ncclAllReduce(bufs[0], bufs[0], count * 2, type(), ncclSum, comm, sh[0].c().stream));
      return nullptr;
    }
    if (!comms.empty()) {
      QDC_NCCL(ncclGroupStart());
      for (size_t s = 0; s < sh.size(); ++s)
        QDC_NCCL(ncclAllReduce(bufs[s], bufs[s], count * 2, type(), ncclSum, comms[s],
                               sh[s].c().stream));
      QDC_NCCL(ncclGroupEnd());
      return nullptr;
    }
    if (multi_stream) QDC_TRY(join(sh));
    Ctx& c0 = sh[0].c();
    QDC_TRY(c0.use());
    for (int s = 1; s < nlocal; ++s) QDC_TRY(elementwise_count<2>(c0, bufs[s], bufs[0], count));
    for (int s = 1; s < nlocal; ++s)
      QDC_HIP(hipMemcpyAsync(bufs[s], bufs[0], count * sizeof(cx), hipMemcpyDeviceToDevice,
                             c0.stream));
    if (multi_stream) QDC_TRY(join(sh));
    return nullptr;
  }
  void destroy() {
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
    for (auto c : comms) (void)ncclCommDestroy(c);
    comms.clear();
  }
};

struct Circuit {
  uint32_t n = 0;   // logical qubits
  uint32_t g = 0;   // rank bits
  uint32_t nl = 0;  // local qubits of a shard
  // interleaved state pair (unsharded): fwd and bwd alternate in 2^gap_bits-chunk blocks of one
  // allocation; chunk c of either state at c + (c & gm), bwd = fwd + 2^gap_bits chunks
  uint32_t gap_bits = 0;
  uint64_t gm = 0;
  std::vector<std::unique_ptr<DevRes>> devs;  // per-device resources (sh[s].d points here)
  Exchange ex;
  std::vector<Shard> sh;
  QubitMap layout;  // physical layout of every shard's `state` (identity until a remap)
  size_t dens_cap = 0, grads_cap = 0;
  cx* host_out = nullptr;  // pinned
  size_t host_cap = 0;
  std::vector<Instr> ins;
  // fused multi-gate passes
  int fuse = 1;             // 0: one HBM pass per gate
  uint32_t fuse_max_ops = FMAX_OPS;
  uint32_t fuse_lcmin = 3;  // min contiguous chunk bits of a fused tile (128-B rows)
  int fuse_meas = 1;        // densities / cotangent injections join fused passes
  int use_rq = 1;           // f32 gate passes run register-resident (qdc_rq.hpp)
  int rq_stats = 0;
  // host time of the calls (qdc_circuit_host_times): per direction (0 run/forward, 1 backward)
  // the calls and the milliseconds of setup, scheduling, program build, launching and the
  // finish (stream sync and result copies), accumulated since the last reset
  double host_ms[2][6] = {};
  using hclock = std::chrono::steady_clock;
  static double ms_between(hclock::time_point a, hclock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  }
  void host_record(int dir, const hclock::time_point (&t)[6]) {
    host_ms[dir][0] += 1;
    for (int k = 1; k < 6; ++k) host_ms[dir][k] += ms_between(t[k - 1], t[k]);
  }
  int rq_prefetch = 1;      // one-state register-resident passes prefetch the next tile (QDC_RQ_PF)
  int rq_prefetch2 = 0;     // two-state ones too (QDC_RQ_PF2; 2 waves/SIMD, measured slower)
  int rq64 = 1;  // f64 gate passes register-resident too (k_rw; QDC_RQ64)
  int rq_slots5 = 1;  // two-state f32 k_rw passes plan five register slots (QDC_RQ_SLOTS5)
  // one-state f32 passes on 2^12 tiles run on two-wave, five-slot, prefetching k_rw tiles
  // instead of four-wave, four-slot k_rq ones (QDC_RQ_FWD5)
  int rq_fwd5 = 0;  // measured 4 % slower per pass (r3i): 16 KiB of LDS per wave caps it at 2 waves/SIMD
  bool rq5() const { return rq_slots5 != 0 && (rq_wave & 1) && !(rq_wave & 4); }
  // one-state one-wave five-slot passes (2^11 tiles, QDC_RW bit 1) prefetch the next tile
  // (QDC_RW bit 3, with QDC_RQ_PF)
  bool rw1_prefetch() const { return (rq_wave & 8) && rq_prefetch; }
  // register-resident tile order: 0 block-contiguous, 1 grid-strided, 2 block-contiguous in
  // XCD-aware block order (QDC_RQ_ORDER).  C2 n = 28, same box (profiles/r5/r5q_*): 2 is
  // +0.4-0.6 % over 0, 1 (concurrent tiles neighbours in memory) -6.5 %
  int rq_order = 2;
  // register-resident passes as straight-line kernels specialized per pass program
  // (qdc_spec.hpp, qdc_jit.hpp; QDC_SPEC): 0 off, 1 for states of >= spec_min_qubits local
  // qubits, 2 always; a call whose program needs more than spec_max distinct kernels runs generic
  int spec_mode = 1;
  uint32_t spec_min_qubits = 22;
  uint32_t spec_max = 160;
  int spec_fwd = 1;  // forward (one-state) passes too (QDC_SPEC_FWD)
  // a program with more than spec_max distinct kernels: its missing kernels are compiled by the
  // JIT's background thread while the generic kernels run its passes, later calls launch the
  // specialized ones as their objects appear (QDC_SPEC_ASYNC=0: such programs stay generic).
  // f32 only by default: f32 specialized and generic passes are bit-identical, so a result never
  // depends on how far the background compiler has got; f64 ones differ in the last bits (the
  // compiler contracts the scalar complex arithmetic differently), so a deep f64 program stays
  // generic — reproducible from call to call — unless QDC_SPEC_ASYNC=1 opts in
  int spec_async = sizeof(real) == 4 ? 1 : 0;
  // generated kernels by pass program (key: qdc_circuit build_program), with their functions
  std::map<std::vector<uint32_t>, SpecEntry> spec_cache;
  uint64_t spec_epoch = 0;
  int rq_wave = 1;  // one wave per register-resident tile (k_rw; QDC_RW bit 0 two-state, bit 1
                    // one-state, bit 2 two-state with the next tile prefetched into AGPRs)
  int rq_permute = 1;       // gate-only passes permute their tile's qubits (QDC_RQ_PERM)
  int rq_perm_shard = 1;    // ... on sharded circuits too (QDC_RQ_PERM_SHARD)
  int rq_grad32 = 1;        // two-state passes hold up to FMAX_GRAD_RQ Gamma stages (QDC_RQ_GRAD32)
  int rq_maxcl = 1;         // relayouts chosen by max closure, else greedily (QDC_RQ_MAXCL)
  uint32_t rq_perm_low = 0;  // low positions a permuting pass fills, 0: default (QDC_RQ_PERM_LOW)
  int rq_gstage = 1;  // two-state passes capped by Gamma stages, not variable gates (QDC_RQ_GSTAGE)
  // one-state fused tile in chunks (QDC_TILE1_CHUNKS): TILE_CHUNKS_1, or TILE_CHUNKS_2 (f32: 2^11
  // amplitudes, one wave per tile on k_rw with five slots when QDC_RW bit 1 is set)
  uint32_t tile1_chunks = TILE_CHUNKS_1;
  // runs of cotangent injections whose cotangents are all diagonal become one elementwise pass
  // (k_diag_inject; QDC_DIAG_INJECT)
  int diag_inject = 1;
  // the backward's leading diagonal-injection passes launched before its program is built
  // (QDC_EARLY_INJECT)
  int early_inject = 1;
  // read-only passes of one-qubit densities on k_dens1 (register partial sums across a block's
  // tiles, one reduction per block; QDC_DENS1=0: k_fused's per-tile reductions)
  int dens1_kernel = 1;
  int dens_split = 1;  // forward passes hold gates or densities, not both (qdc_fusion.hpp split_dens)
  // Mirrored schedules (QDC_MIRROR): the forward is scheduled on the two-state tile under both
  // directions' rules (qdc_fusion.hpp FusionPlanner::mirror) and the backward runs its passes in
  // reverse, uncomputing each stage with exactly the adjoint of the matrix the forward applied —
  // the O(1)-memory uncompute then drifts like the reference's gate-by-gate U, U^dagger sequence
  // instead of accumulating the rounding of independently formed stage products.  Sharded
  // circuits too (round 5): the forward's remap plan keeps both directions' order relations and
  // the backward undoes its remaps in reverse (unremap).  The backward must follow a forward call
  // with the same gates (else the backward schedules itself as usual).  On by default (round 4: C5 n = 14 f32 uncompute 4.85x -> 1.4x
  // the reference's floor; C2 n = 28 f32 ~3.5 % slower, DESIGN.md "Uncompute drift").
  int mirror = 1;
  // one-state one-wave specialized passes relayout through half the LDS buffer when every
  // relayout keeps a register slot (QDC_SPEC_HALF; twice the resident waves)
  int spec_half = 1;
  // trailing one-qubit stages of a pass join their qubit's next two-qubit stage in a later pass
  // (qdc_fusion.hpp defer_trailing_q1; QDC_DEFER_Q1)
  int defer_q1 = 1;
  bool mirror_on() const {
    return mirror && fuse && fuse_max_ops >= 2 && use_rq && (sizeof(real) == 4 || rq64);
  }
  // one-state one-wave five-slot passes on 2^11 tiles (f32): QDC_RW bit 1, or a mirrored forward
  bool rw1() const { return (rq_wave & 2) || mirror_on(); }

  // host-only dry run (init_dry): calls stop before their first launch; build_program writes
  // the pass program into dry_prog and collects the specialized kernels into dry_specs
  bool dry = false;
  std::vector<unsigned char> dry_prog;
  std::vector<SpecEntry*> dry_specs;
  // dry-run trace of the matrices a call applies to the forward state (qdc_trace_program, the
  // host emulation tools/drift_emu.py): per fused stage or single gate its logical qubits (row
  // index 2 bit(q2) + bit(q1); q2 == q1 for one qubit), the matrix as uploaded (working
  // precision, diagonals expanded) and whether it is the adjoint of a recorded forward matrix
  struct TraceOp {
    uint32_t dir, item, q2, q1, R, diag, mirrored, single;
    qdc_complex m[16];
  };
  bool tracing = false;
  std::vector<TraceOp> trace;
  size_t trace_from = 0;
  std::vector<uint8_t> inexact;  // per instruction: gate not unitary to working precision
  uint32_t fused_blocks = 0;  // 0: as many blocks as are resident at once (occupancy query)
  std::vector<std::pair<const void*, uint32_t>> fused_resident_cache;
  uint32_t last_fused_grid = 0;
  uint32_t last_fused_ndyn = 0;  // granule partials per slot of the last fused launch
  unsigned char* prog_host = nullptr;  // pinned staging of the pass program (every device's copy)
  std::vector<StagePost> stage_post;   // gradient recipes of the last backward's stages
  size_t prog_cap = 0;

  Ctx& ctx0() { return devs[0]->ctx; }
  const char* sync_all() {
    for (auto& d : devs) QDC_TRY(d->ctx.sync());
    return nullptr;
  }
  const char* flush_all() {  // pending reduction slots of every context
    for (auto& d : devs) {
      QDC_TRY(d->ctx.use());
      QDC_TRY(d->ctx.flush());
    }
    return nullptr;
  }

  // world = total shards (power of two), nlocal = shards in this process.  devices: one device
  // per local shard, each shard on its own stream (nullptr: every local shard on the current
  // device and one stream).  comms: one RCCL communicator per local shard (ncclCommInitAll;
  // devices then distinct), or none (copies between the streams of one device).
  const char* init(uint32_t qubits, int world = 1, int rank0 = 0, int nlocal = 1,
                   ncclComm_t comm = nullptr, const std::vector<int>* devices = nullptr,
                   const std::vector<ncclComm_t>* comms = nullptr) {
    DeviceGuard keep;
    // the communicators are owned from here on (destroy() frees them, also on a failure below)
    if (comms) ex.comms = *comms;
    n = qubits;
    const uint32_t gg = log2_exact((size_t)world);
    if (gg == UINT32_MAX || gg > 8) return fail("the number of shards must be a power of two <= 256");
    g = gg;
    if (g > 0 && n < 2 * g + 3)
      return fail("%u qubits are too few to shard over %d ranks (need >= %u)", n, world, 2 * g + 3);
    nl = n - g;
    ex.world = world;
    ex.rank0 = rank0;
    ex.nlocal = nlocal;
    ex.comm = comm;
    ex.multi_stream = devices != nullptr && ex.comms.empty() && nlocal > 1;
    layout.identity(n, g);
    QDC_TRY(read_knobs(world, nlocal));
    int cur = 0;
    QDC_HIP(hipGetDevice(&cur));
    const int ndev = devices ? nlocal : 1;
    for (int i = 0; i < ndev; ++i) {
      devs.push_back(std::make_unique<DevRes>());
      QDC_TRY(devs.back()->ctx.init(devices ? (*devices)[i] : cur));
    }
    const size_t bytes = ((size_t)1 << nl) * sizeof(cx);
    sh.resize(nlocal);
    for (int s = 0; s < nlocal; ++s) {
      sh[s].d = devs[devices ? s : 0].get();
      Ctx& c = sh[s].c();
      QDC_TRY(c.use());
      QDC_HIP(hipMalloc(&sh[s].initial, bytes));
      sh[s].owned.push_back(sh[s].initial);
      QDC_TRY(alloc_pair(sh[s], bytes));
      if (g > 0) {
        QDC_HIP(hipMalloc(&sh[s].scratch, bytes));
        sh[s].owned.push_back(sh[s].scratch);
      }
      // QuantizedTensor::new_standard + clone (circuit.rs:96-102): |0..0> lives on shard 0
      if (rank0 + s == 0)
        QDC_TRY(set_standard(c, sh[s].initial, nl));
      else
        QDC_HIP(hipMemsetAsync(sh[s].initial, 0, bytes, c.stream));
      QDC_TRY(copy_initial(sh[s]));
    }
    QDC_TRY(sync_all());
    return nullptr;
  }
  // the runtime's QDC_* knobs (environment, read once per circuit)
  const char* read_knobs(int world, int nlocal) {
    if (const char* e = getenv("QDC_FUSE")) fuse = atoi(e);
    if (const char* e = getenv("QDC_FUSE_MAX_OPS"))
      fuse_max_ops = std::max(1, std::min(atoi(e), FMAX_OPS));
    if (const char* e = getenv("QDC_FUSE_MEAS")) fuse_meas = atoi(e);
    if (const char* e = getenv("QDC_RQ")) use_rq = atoi(e);
    if (const char* e = getenv("QDC_RQ_STATS")) rq_stats = atoi(e);
    if (const char* e = getenv("QDC_RQ_PF")) rq_prefetch = atoi(e);
    if (const char* e = getenv("QDC_RQ_PF2")) rq_prefetch2 = atoi(e);
    if (const char* e = getenv("QDC_RW")) rq_wave = atoi(e);
    if (const char* e = getenv("QDC_RQ_ORDER")) rq_order = atoi(e);
    if (const char* e = getenv("QDC_RQ64")) rq64 = atoi(e);
    if (const char* e = getenv("QDC_RQ_SLOTS5")) rq_slots5 = atoi(e);
    if (const char* e = getenv("QDC_RQ_FWD5")) rq_fwd5 = atoi(e);
    if (const char* e = getenv("QDC_RQ_PERM")) rq_permute = atoi(e);
    if (const char* e = getenv("QDC_RQ_PERM_SHARD")) rq_perm_shard = atoi(e);
    if (const char* e = getenv("QDC_RQ_GRAD32")) rq_grad32 = atoi(e);
    if (const char* e = getenv("QDC_RQ_MAXCL")) rq_maxcl = atoi(e);
    if (const char* e = getenv("QDC_RQ_PERM_LOW")) rq_perm_low = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_RQ_GSTAGE")) rq_gstage = atoi(e);
    if (const char* e = getenv("QDC_DIAG_INJECT")) diag_inject = atoi(e);
    if (const char* e = getenv("QDC_EARLY_INJECT")) early_inject = atoi(e);
    if (const char* e = getenv("QDC_DENS1")) dens1_kernel = atoi(e);
    if (const char* e = getenv("QDC_DENS_SPLIT")) dens_split = atoi(e);
    if (const char* e = getenv("QDC_MIRROR")) mirror = atoi(e);
    if (const char* e = getenv("QDC_SPEC_HALF")) spec_half = atoi(e);
    if (const char* e = getenv("QDC_DEFER_Q1")) defer_q1 = atoi(e);
    if (const char* e = getenv("QDC_SCHED_CACHE")) sched_cache_on = atoi(e);
    if (const char* e = getenv("QDC_TILE1_CHUNKS")) {
      const uint32_t t = (uint32_t)atoi(e);
      if (t != TILE_CHUNKS_1 && t != TILE_CHUNKS_2)
        return fail("QDC_TILE1_CHUNKS must be %u or %u", TILE_CHUNKS_1, TILE_CHUNKS_2);
      tile1_chunks = t;
    }
    if (const char* e = getenv("QDC_SPEC")) spec_mode = atoi(e);
    if (const char* e = getenv("QDC_SPEC_MIN_QUBITS")) spec_min_qubits = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_SPEC_MAX")) spec_max = (uint32_t)atoi(e);
    if (const char* e = getenv("QDC_SPEC_FWD")) spec_fwd = atoi(e);
    if (const char* e = getenv("QDC_SPEC_ASYNC")) spec_async = atoi(e);
    // the node's hipcc processes shared among the ranks of a multi-process job
    SpecJit::get().set_processes(std::max(1, world / std::max(1, nlocal)));

    if (const char* e = getenv("QDC_FUSE_LCMIN"))
      fuse_lcmin = (uint32_t)std::max(1, std::min(atoi(e), LOWBITS));
    if (const char* e = getenv("QDC_FUSED_BLOCKS"))
      fused_blocks = (uint32_t)std::max(1, std::min(atoi(e), (int)NBMAX));
    return nullptr;
  }
  // A host-only circuit (no device, no state): plans, schedules and pass programs exactly as
  // execute() / backward() build them, for the specialized kernels compiled ahead of time
  // (qdc_precompile; dry-run calls return before their first launch).
  const char* init_dry(uint32_t qubits, int world) {
    dry = true;
    n = qubits;
    const uint32_t gg = log2_exact((size_t)world);
    if (gg == UINT32_MAX || gg > 8) return fail("the number of shards must be a power of two <= 256");
    g = gg;
    if (g > 0 && n < 2 * g + 3)
      return fail("%u qubits are too few to shard over %d ranks (need >= %u)", n, world, 2 * g + 3);
    nl = n - g;
    ex.world = world;
    ex.nlocal = 1;
    layout.identity(n, g);
    return read_knobs(world, world);  // (compiles: this process's full parallelism)
  }
  void destroy() {
    DeviceGuard keep;
    (void)sync_all();
    for (auto& s : sh) {
      if (s.d) (void)s.d->ctx.use();
      for (void* p : s.owned) (void)hipFree(p);
      for (cx* p : {s.dens, s.grads})
        if (p) (void)hipFree(p);
    }
    sh.clear();
    if (host_out) (void)hipHostFree(host_out);
    host_out = nullptr;
    for (auto& d : devs) {
      (void)d->ctx.use();
      if (d->prog_dev) (void)hipFree(d->prog_dev);
      d->prog_dev = nullptr;
      d->ctx.destroy();
    }
    devs.clear();
    if (prog_host) (void)hipHostFree(prog_host);
    prog_host = nullptr;
    ex.destroy();
  }

  // The forward and cotangent states as one allocation, interleaved in 64 KiB blocks (chunk
  // bit 12 selects the state).  Two states streamed together then run at one steady rate
  // whatever the placement (6.5 TB/s for in-place fwd+bwd at n = 28), while two separate 2 GiB
  // allocations land on placements that stream at 5.0-6.5 TB/s and the single-gate reverse
  // kernels at 64 % or 79 % of 8 TB/s from one circuit to the next (tools/alloc_probe.hip,
  // tools/pair_probe.hip, profiles/r2e_*, r2f_*).  Unsharded circuits only (a remap swaps the
  // states with the scratch buffer); QDC_STATE_ILV=0 keeps the plain layout (bwd separate and
  // allocated on the first backward).  The initial copy, the bwd zeroing and every gate-shaped
  // kernel address the pair through Ctx::gm; readbacks copy block by block (read_state).
  const char* alloc_pair(Shard& s, size_t bytes) {
    const char* e = getenv("QDC_STATE_ILV");
    // block size: 2^12 chunks (QDC_STATE_ILV_BITS); states of at least two blocks
    uint32_t gb = 12;
    if (const char* b = getenv("QDC_STATE_ILV_BITS")) gb = (uint32_t)std::max(4, std::min(atoi(b), 24));
    bool ilv = !(e && atoi(e) == 0) && g == 0 && sh.size() == 1 &&
               nchunks_of(nl) >= ((uint64_t)2 << gb);
    if (ilv) {
      // the pair allocates bwd now, not on the first backward (circuit.rs:276 creates it
      // lazily): when the device cannot hold it beside `initial` plus 1 GiB of headroom, keep
      // the plain layout, so a run/forward-only circuit still needs only two states
      size_t free_b = 0, total_b = 0;
      QDC_HIP(hipMemGetInfo(&free_b, &total_b));
      if (free_b < 2 * bytes + ((size_t)1 << 30)) ilv = false;
    }
    if (ilv) {
      gap_bits = gb;
      gm = ~(((uint64_t)1 << gap_bits) - 1);
      char* blk = nullptr;
      QDC_HIP(hipMalloc(&blk, 2 * bytes));
      s.owned.push_back(blk);
      s.state = (cx*)blk;
      s.bwd = (cx*)blk + ((size_t)VEC << gap_bits);
      s.c().gm = gm;
    } else {
      QDC_HIP(hipMalloc(&s.state, bytes));
      s.owned.push_back(s.state);
    }
    return nullptr;
  }
  // (kernels: a 2-D hipMemset / hipMemcpy over the 64 KiB blocks runs at < 1 TB/s)
  // every call starts from `initial`; while that is the standard state (the reference's
  // new_standard, circuit.rs:96-102: no set_state_from_vector yet) the state is written directly
  // (|0..0> on shard 0, zeros elsewhere: one write of S instead of a copy's read and write)
  bool initial_standard = true;
  const char* copy_initial(Shard& s) {
    if (initial_standard) {
      const bool first = ex.rank0 + (int)(&s - sh.data()) == 0;
      return first ? elementwise<3>(s.c(), nullptr, s.state, nl, gm)
                   : elementwise<4>(s.c(), nullptr, s.state, nl, gm);
    }
    return elementwise<0>(s.c(), s.initial, s.state, nl, gm);
  }
  const char* zero_bwd(Shard& s) {
    if (gm) return elementwise<4>(s.c(), nullptr, s.bwd, nl, gm);
    QDC_HIP(hipMemsetAsync(s.bwd, 0, ((size_t)1 << nl) * sizeof(cx), s.c().stream));
    return nullptr;
  }
  // host copy of amplitudes [offset, offset + len) of a (possibly interleaved) state
  const char* read_state(const Shard& s, const cx* src, size_t offset, qdc_complex* host,
                         size_t len) {
    const hipStream_t st = s.c().stream;
    if (!gm || (src != s.state && src != s.bwd)) {
      QDC_HIP(hipMemcpyAsync(host, src + offset, len * sizeof(cx), hipMemcpyDeviceToHost, st));
      return nullptr;
    }
    const size_t row = (size_t)VEC << gap_bits;  // amplitudes per block
    size_t o = offset, done = 0;
    auto piece = [&](size_t cnt) -> const char* {  // within one block
      const size_t phys = (o / row) * 2 * row + o % row;
      QDC_HIP(hipMemcpyAsync(host + done, src + phys, cnt * sizeof(cx), hipMemcpyDeviceToHost, st));
      o += cnt;
      done += cnt;
      return nullptr;
    };
    if (o % row && done < len) QDC_TRY(piece(std::min(len - done, row - o % row)));
    const size_t full = (len - done) / row;
    if (full) {
      QDC_HIP(hipMemcpy2DAsync(host + done, row * sizeof(cx), src + (o / row) * 2 * row,
                               2 * row * sizeof(cx), row * sizeof(cx), full,
                               hipMemcpyDeviceToHost, st));
      o += full * row;
      done += full * row;
    }
    if (done < len) QDC_TRY(piece(len - done));
    return nullptr;
  }

  const char* ensure_out(bool dens, size_t count) {
    size_t& cap = dens ? dens_cap : grads_cap;
    if (count <= cap) return nullptr;
    QDC_TRY(sync_all());
    for (auto& s : sh) {
      QDC_TRY(s.c().use());
      cx*& p = dens ? s.dens : s.grads;
      if (p) QDC_HIP(hipFree(p));
      p = nullptr;
      QDC_HIP(hipMalloc(&p, sizeof(cx) * count));
    }
    cap = count;
    return nullptr;
  }
  const char* ensure_host(size_t count) {
    if (count <= host_cap) return nullptr;
    if (host_out) {
      QDC_TRY(sync_all());
      QDC_HIP(hipHostFree(host_out));
    }
    host_out = nullptr;
    QDC_HIP(hipHostMalloc(&host_out, sizeof(cx) * count));
    host_cap = count;
    return nullptr;
  }

  size_t output_count(int mode) const {
    size_t c = 0;
    for (auto& in : ins)
      if (is_diff_density(in.kind) || (mode == QDC_MODE_RUN && is_density(in.kind))) ++c;
    return c;
  }
  size_t output_size(int mode) const {
    size_t c = 0;
    for (auto& in : ins)
      if (is_diff_density(in.kind) || (mode == QDC_MODE_RUN && is_density(in.kind)))
        c += is_q1_density(in.kind) ? 4 : 16;
    return c;
  }
  size_t n_var() const {
    size_t c = 0;
    for (auto& in : ins) c += is_var(in.kind);
    return c;
  }
  size_t grad_size() const {
    size_t c = 0;
    for (auto& in : ins)
      if (is_var(in.kind)) c += gate_len(in.kind);
    return c;
  }

  // --- validation: the reference's panic order (circuit.rs:170-211, 221-263, 274-428) --------
  const char* validate_forward(const Flat& cg, const Flat& vg, std::vector<size_t>& gidx) const {
    if (ins.empty()) return fail("The circuit is empty.");
    size_t ci = 0, vi = 0;
    gidx.assign(ins.size(), 0);
    for (size_t k = 0; k < ins.size(); ++k) {
      const Instr& in = ins[k];
      if (is_const(in.kind)) {
        if (ci >= cg.size()) return fail("The number of constant gates is less than required.");
        gidx[k] = ci;
        QDC_TRY(check_gate(in, cg.len[ci], n));
        ++ci;
      } else if (is_var(in.kind)) {
        if (vi >= vg.size()) {
          // circuit.rs:198 / :249 report the constant-gate message for VarQ2GateDiag
          if (in.kind == QDC_VAR_Q2_DIAG)
            return fail("The number of constant gates is less than required.");
          return fail("The number of variable gates is less than required.");
        }
        gidx[k] = vi;
        QDC_TRY(check_gate(in, vg.len[vi], n));
        ++vi;
      } else {
        QDC_TRY(check_density_pos(in, n));
      }
    }
    if (ci != cg.size()) return fail("Number of constant gates is more than required.");
    if (vi != vg.size()) return fail("Number of variable gates is more than required.");
    return nullptr;
  }

  const char* validate_backward(const Flat& dg, const Flat& cg, const Flat& vg,
                                std::vector<size_t>& gidx) const {
    if (ins.empty()) return fail("The circuit is empty.");
    size_t ci = cg.size(), vi = vg.size(), di = dg.size();
    gidx.assign(ins.size(), 0);
    for (size_t kk = ins.size(); kk-- > 0;) {
      const Instr& in = ins[kk];
      if (is_const(in.kind)) {
        if (ci == 0) return fail("The number of gates is less than required.");
        --ci;
        gidx[kk] = ci;
        QDC_TRY(check_gate(in, cg.len[ci], n));
      } else if (is_var(in.kind)) {
        if (vi == 0) return fail("The number of gates is less than required.");
        --vi;
        gidx[kk] = vi;
        QDC_TRY(check_gate(in, vg.len[vi], n));
      } else if (is_diff_density(in.kind)) {
        if (di == 0)
          return fail("The number of gradients wrt density matrices is less than required.");
        --di;
        gidx[kk] = di;
        const size_t want = is_q1_density(in.kind) ? 4 : 16;
        if (dg.len[di] != want) return fail("Incorrect len of the gate's buffer.");
        QDC_TRY(check_density_pos(in, n));
      }
    }
    if (ci != 0) return fail("Number of constant gates is more than required.");
    // circuit.rs:426 reports leftover variable gates with the constant-gate message
    if (vi != 0) return fail("Number of constant gates is more than required.");
    if (di != 0)
      return fail("Number of gradients wrt density matrices is more than required.");
    return nullptr;
  }

  // --- remap: one all-to-all per state (see qdc_shard.hpp) --------------------------------
  const char* remap(const qdc_plan_op& r, bool with_bwd) {
    const uint32_t low = nl - g;              // amplitude bits of one all-to-all block
    const size_t chunk = (size_t)1 << low;    // amplitudes per block
    for (int which = 0; which < (with_bwd ? 2 : 1); ++which) {
      std::vector<cx*> send(sh.size()), recv(sh.size());
      for (size_t s = 0; s < sh.size(); ++s) {
        cx*& buf = which == 0 ? sh[s].state : sh[s].bwd;
        if (r.pack) {
          QDC_TRY(sh[s].c().use());
          QDC_TRY(pack(sh[s].c(), buf, sh[s].scratch, r.victims, g, nl));
          send[s] = sh[s].scratch;
          recv[s] = buf;
        } else {
          send[s] = buf;
          recv[s] = sh[s].scratch;
        }
      }
      QDC_TRY(ex.alltoall(sh, send, recv, chunk));
      if (!r.pack)
        for (size_t s = 0; s < sh.size(); ++s)
          std::swap(which == 0 ? sh[s].state : sh[s].bwd, sh[s].scratch);
    }
    layout.apply(r.victims);
    return nullptr;
  }
  // The inverse of remap(r): the all-to-all first (its block exchange, block j of shard s <->
  // block s of shard j, is its own inverse), then the pack's inverse permutation.  A mirrored
  // reverse sweep undoes the forward's remaps in reverse order, so each of its passes finds the
  // physical layout its forward pass ran in.
  const char* unremap(const qdc_plan_op& r, bool with_bwd) {
    const uint32_t low = nl - g;
    const size_t chunk = (size_t)1 << low;
    for (int which = 0; which < (with_bwd ? 2 : 1); ++which) {
      std::vector<cx*> send(sh.size()), recv(sh.size());
      for (size_t s = 0; s < sh.size(); ++s) {
        send[s] = which == 0 ? sh[s].state : sh[s].bwd;
        recv[s] = sh[s].scratch;
      }
      QDC_TRY(ex.alltoall(sh, send, recv, chunk));
      for (size_t s = 0; s < sh.size(); ++s) {
        cx*& buf = which == 0 ? sh[s].state : sh[s].bwd;
        if (r.pack) {
          QDC_TRY(sh[s].c().use());
          QDC_TRY(pack(sh[s].c(), sh[s].scratch, buf, r.victims, g, nl, true));
        } else {
          std::swap(buf, sh[s].scratch);
        }
      }
    }
    layout.unapply(r.victims);
    return nullptr;
  }

  std::vector<qdc_plan_op> plan(int mode) const {
    std::vector<PlanIn> ops;
    std::vector<int> index;
    active_ops(ins, mode, ops, index);
    QubitMap m = layout;
    std::vector<qdc_plan_op> out;
    // a mirrored forward's remap plan keeps both directions' order relations (its reverse is
    // the backward's plan)
    plan_pass(ops, index, m, out, mode == QDC_PLAN_BACKWARD, &inexact,
              mode == QDC_PLAN_FORWARD && mirror_on());
    return out;
  }

  struct Item : FusionItem {
    std::vector<std::vector<uint32_t>> stages;  // fused pass: its stages (stage_partition)
    // a mirrored backward pass: per stage the forward (item, stage) it undoes
    std::vector<std::pair<uint32_t, uint32_t>> mirror_of;
    size_t fop_off = 0;  // byte offset of the group's fop array in the pass program
    uint32_t nstage = 0;  // fop count (stages) of the pass
    double flops_per_amp = 0;  // algorithmic real FLOPs per amplitude of the pass
    bool has_red = false;      // reduction ops (Gamma stages or densities)
    bool writes_f = false;     // gate stages (fwd changes; else fwd is only read)
    std::vector<uint32_t> grad_slots;  // reduction slot of each reduction op, in op order
    bool rq = false;   // register-resident pass (qdc_rq.hpp): k_rq, ops include relayouts
    bool s5 = false;   // rq with five register slots (k_rw<true, 2, false, 1, true>)
    bool inv = false;  // a remap (type 1) run backwards: a mirrored backward undoing the forward's remap
    bool dens1 = false;  // a read-only pass of one-qubit densities only: k_dens1
    uint32_t l0 = 0;   // rq: matrix-area offset (cx) of the L0 layout descriptor
    uint32_t tbits = 0;  // amplitude bits of the tile
    // specialized kernel of a five-slot reverse pass or a one-state forward pass (qdc_jit.hpp): name, source, function
    SpecEntry* spec = nullptr;  // specialized kernel of the pass (qdc_jit.hpp), or none
  };
  // what a mirrored backward needs from the forward call: its schedule (plan after the
  // permuting passes' rewrites, items with stages), each gate stage's forward matrix (double,
  // in the forward's frame) and the gates and inexact flags it was built from
  struct MirrorRec {
    bool valid = false;
    std::vector<qdc_plan_op> plan;
    std::vector<Item> items;
    std::vector<std::vector<SMat>> stage_mats;  // [item][stage] (gate stages; else unused)
    std::vector<qdc_complex> cgates, vgates;
    std::vector<uint8_t> inexact;
    std::vector<uint32_t> end_phys;  // the layout the forward left
  } mrec;
  std::vector<std::vector<SMat>>* rec_mats = nullptr;  // build_program records stage matrices here
  // The backward schedule as the forward's passes run in reverse (mirror mode): op positions
  // mapped into the layout each reverse pass starts from (the forward pass's store layout),
  // stages and the ops in them reversed, the forward's swaps undone in reverse order.
  bool mirror_schedule(std::vector<qdc_plan_op>& pl, std::vector<Item>& items,
                       size_t& first_inject) const {
    pl.clear();
    items.clear();
    const std::vector<Item>& F = mrec.items;
    for (size_t k = F.size(); k-- > 0;) {
      const Item& f = F[k];
      if (f.type != 0 && f.type != 1 && f.type != 2) return false;
      auto sigma = [&](uint32_t p) {
        for (const auto& sw : f.swaps) {
          if (p == sw.first) p = sw.second;
          else if (p == sw.second) p = sw.first;
        }
        return p;
      };
      auto push = [&](uint32_t fi) {
        qdc_plan_op op = mrec.plan[fi];
        if (op.type == QDC_PLAN_OP) {
          op.pos2 = sigma(op.pos2);
          op.pos1 = sigma(op.pos1);
        }
        pl.push_back(op);
        return (uint32_t)(pl.size() - 1);
      };
      auto shell = [&]() {
        Item b;
        b.type = 2;
        b.lc = f.lc;
        b.h = f.h;
        for (uint32_t r = 0; r < (uint32_t)FMAX_ROWS; ++r) b.hb[r] = f.hb[r];
        return b;
      };
      if (f.type != 2) {  // a single op, or a remap undone (unremap)
        Item b;
        b.type = f.type;
        b.inv = f.type == 1;
        b.ops.push_back(push(f.ops[0]));
        items.push_back(std::move(b));
        continue;
      }
      // the pass's densities (its last stages) become the injections that open its reverse
      // pass (one injection pass; a single one stays a single op), then its gate stages in
      // reverse with the forward's swaps undone in reverse order
      size_t ng = f.stages.size();
      while (ng > 0 && is_meas(mrec.plan[f.stages[ng - 1][0]])) --ng;
      for (size_t j = ng; j < f.stages.size(); ++j)
        for (uint32_t fi : f.stages[j])
          if (!is_meas(mrec.plan[fi])) return false;  // (the planner keeps densities last)
      if (ng < f.stages.size()) {
        Item m = shell();
        for (size_t j = f.stages.size(); j-- > ng;) {
          const uint32_t bi = push(f.stages[j][0]);
          m.ops.push_back(bi);
          m.stages.push_back({bi});
        }
        if (m.ops.size() == 1) {
          m.type = 0;
          m.stages.clear();
        }
        items.push_back(std::move(m));
      }
      if (ng == 0) continue;
      Item b = shell();
      for (auto it = f.swaps.rbegin(); it != f.swaps.rend(); ++it) b.swaps.push_back(*it);
      for (size_t j = ng; j-- > 0;) {
        std::vector<uint32_t> st;
        for (size_t t = f.stages[j].size(); t-- > 0;) {
          if (is_meas(mrec.plan[f.stages[j][t]])) return false;
          const uint32_t bi = push(f.stages[j][t]);
          st.push_back(bi);
          b.ops.push_back(bi);
        }
        b.stages.push_back(std::move(st));
        b.mirror_of.push_back({(uint32_t)k, (uint32_t)j});
      }
      items.push_back(std::move(b));
    }
    first_inject = pl.size();
    for (size_t i = 0; i < pl.size(); ++i)
      if (pl[i].type == QDC_PLAN_OP && is_diff_density(ins[pl[i].instr].kind)) {
        first_inject = i;
        break;
      }
    return true;
  }
  static constexpr uint32_t TILE_CHUNKS_1 = FusionPlanner::TILE_CHUNKS_1;
  static constexpr uint32_t TILE_CHUNKS_2 = FusionPlanner::TILE_CHUNKS_2;
  FusionPlanner planner() const {
    FusionPlanner P{ins, inexact, nl, fuse != 0, fuse_meas != 0, fuse_max_ops, fuse_lcmin};
    // gate-only passes permute their tile on the way out when they are register-resident
    // (sharded circuits too, round 5: later remaps' victims are relabelled, qdc_fusion.hpp
    // relabel_remap; QDC_RQ_PERM_SHARD=0 keeps their layouts fixed)
    P.permute = rq_permute && use_rq && (g == 0 || rq_perm_shard) && sizeof(real) == 4;
    P.ng = g;
    P.rq_grad = rq_grad32 && use_rq && (sizeof(real) == 4 || rq64);
    if (rq_perm_low) P.perm_low = rq_perm_low;
    P.tile1_chunks = tile1_chunks;
    P.mirror = mirror_on() && sched_mirror;
    P.defer_q1 = defer_q1 != 0;
    P.gamma_stage_cap = rq_gstage != 0;
    P.split_dens = dens_split != 0;
    return P;
  }
  bool is_meas(const qdc_plan_op& op) const { return planner().is_meas(op); }
  std::vector<Item> fuse_items(std::vector<qdc_plan_op>& plan, bool backward,
                               size_t first_inject = SIZE_MAX) const {
    std::vector<Item> items;
    for (FusionItem& f : planner().fuse_items(plan, backward, first_inject)) {
      Item it;
      static_cast<FusionItem&>(it) = std::move(f);
      if (it.type == 2) it.stages = stage_partition(it.ops, plan, backward);
      items.push_back(std::move(it));
    }
    return items;
  }
  // The pass schedule of a call (fuse_items + stage_partition, ~1-2 ms at C2 n = 28) depends on
  // the plan, the inexact flags and the mode only, not on the gate values: the last schedule
  // per direction is kept and reused when those are unchanged (QDC_SCHED_CACHE=0: off).
  struct SchedCache {
    bool valid = false;
    size_t first_inject = 0;
    bool mirror = false;
    std::vector<qdc_plan_op> in_plan, out_plan;
    std::vector<uint8_t> inexact;
    std::vector<Item> items;
  };
  SchedCache sched_cache[2];  // forward / run, backward
  // the schedule being built is a mirrored forward's (forward calls only: a run call has no
  // backward to mirror and keeps the one-state schedule)
  bool sched_mirror = false;
  int sched_cache_on = 1;
  static bool same_plan(const std::vector<qdc_plan_op>& a, const std::vector<qdc_plan_op>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
      const qdc_plan_op &x = a[i], &y = b[i];
      if (x.type != y.type || x.instr != y.instr || x.pos2 != y.pos2 || x.pos1 != y.pos1 ||
          x.nvictims != y.nvictims || x.pack != y.pack)
        return false;
      for (unsigned k = 0; k < x.nvictims && k < 8; ++k)
        if (x.victims[k] != y.victims[k]) return false;
    }
    return true;
  }
  std::vector<Item> schedule(std::vector<qdc_plan_op>& plan, bool backward, size_t first_inject) {
    SchedCache& c = sched_cache[backward ? 1 : 0];
    if (sched_cache_on && c.valid && c.first_inject == first_inject && c.inexact == inexact &&
        c.mirror == sched_mirror && same_plan(c.in_plan, plan)) {
      plan = c.out_plan;
      return c.items;
    }
    c.valid = false;
    c.in_plan = plan;
    std::vector<Item> items = fuse_items(plan, backward, first_inject);
    if (sched_cache_on) {
      c.out_plan = plan;
      c.items = items;
      c.inexact = inexact;
      c.first_inject = first_inject;
      c.mirror = sched_mirror;
      c.valid = true;
    }
    return items;
  }
  // register-layout plans of passes (rq_plan, ~20 us each), by the pass's stages and tile
  std::map<std::vector<uint64_t>, RqPlan> rq_plan_cache;
  const RqPlan& rq_plan_cached(const std::vector<RqStage>& rs, uint32_t tbits, const uint32_t* src,
                               bool maxcl, uint32_t ns, bool keep = false) {
    std::vector<uint64_t> key = {tbits, ns, (maxcl ? 1u : 0u) | (keep ? 2u : 0u), src ? 1u : 0u};
    if (src)
      for (int i = 0; i < 4; ++i) key.push_back(src[i]);
    for (const RqStage& r : rs) {
      key.push_back(((uint64_t)r.kind << 48) | ((uint64_t)r.t1 << 24) | r.t2);
      key.push_back(r.deps);
    }
    auto it = rq_plan_cache.find(key);
    if (it != rq_plan_cache.end()) return it->second;
    if (rq_plan_cache.size() >= 8192) rq_plan_cache.clear();
    return rq_plan_cache.emplace(std::move(key), rq_plan(rs, tbits, src, maxcl, ns, keep)).first->second;
  }
  std::vector<std::vector<uint32_t>> stage_partition(const std::vector<uint32_t>& pass,
                                                     const std::vector<qdc_plan_op>& plan,
                                                     bool backward) const {
    return planner().stage_partition(pass, plan, backward);
  }
  // per call: which gates are not unitary to working precision (qdc_fusion.hpp)
  void mark_inexact(const Flat& cg, const Flat& vg, const std::vector<size_t>& gidx) {
    inexact.assign(ins.size(), 0);
    const double utol = sizeof(real) == 4 ? 1e-6 : 1e-13;
    for (size_t k = 0; k < ins.size(); ++k)
      if (is_const(ins[k].kind) || is_var(ins[k].kind)) {
        const qdc_complex* g4 = is_const(ins[k].kind) ? cg.at(gidx[k]) : vg.at(gidx[k]);
        inexact[k] = unitarity_error(g4, ins[k].kind) > utol ? 1 : 0;
      }
  }
  // max |U^+ U - I| of a gate's host matrix (diagonal: max ||d_i|^2 - 1|)
  static double unitarity_error(const qdc_complex* g, int kind) {
    if (is_diag(kind)) {
      double e = 0;
      for (int i = 0; i < 4; ++i) {
        const double m = (double)g[i].re * g[i].re + (double)g[i].im * g[i].im;
        e = std::max(e, std::abs(m - 1.0));
      }
      return e;
    }
    const int R = is_q1_gate(kind) ? 2 : 4;
    double e = 0;
    for (int p = 0; p < R; ++p)
      for (int q = 0; q < R; ++q) {
        double re = 0, im = 0;  // (U^+ U)[p][q] = sum_k conj(U[k][p]) U[k][q]
        for (int k = 0; k < R; ++k) {
          const qdc_complex a = g[k * R + p], b = g[k * R + q];
          re += (double)a.re * b.re + (double)a.im * b.im;
          im += (double)a.re * b.im - (double)a.im * b.re;
        }
        e = std::max(e, std::hypot(re - (p == q ? 1.0 : 0.0), im));
      }
    return e;
  }
  // Lay out every fused pass's stage descriptors and stage matrices (A = product of the
  // applied matrices, B = product of the bwd pull-backs) in one pinned buffer, then upload it.
  // backward: `first_inject` = plan index of the first cotangent injection (passes before it
  // only uncompute fwd); gradient stages get slots nvar, nvar+1, ... of the gradient buffer and
  // a recipe in stage_post (qdc_stage.hpp).
  // forward: densities reduce into dens slot out_idx[instr]; backward: injections read their
  // cotangent from dg.
  const char* build_program(std::vector<Item>& items, const std::vector<qdc_plan_op>& plan,
                            bool backward, size_t first_inject, const Flat& cg, const Flat& vg,
                            const std::vector<size_t>& gidx, size_t& mats_off,
                            const std::vector<uint32_t>& var_idx, uint32_t nvar,
                            const std::vector<uint32_t>& out_idx, const Flat* dg) {
    stage_post.clear();
    if (spec_cache.size() >= 4096 && !dry) spec_cache.clear();  // bounded; items of this call point into it
    size_t nops = 0;
    for (size_t ii = 0; ii < items.size(); ++ii)
      if (items[ii].type == 2) nops += items[ii].stages.size();
    if (nops == 0) return nullptr;
    // register-resident passes add relayout ops (<= one per stage, plus the return to L0) and
    // 12-cx layout descriptors (one per relayout, plus L0)
    const size_t nfops = 2 * nops + items.size();
    mats_off = ((nfops * sizeof(fop) + 255) / 256) * 256;
    // matrices <= 2 R^2 = 32 per stage; layouts <= 12 cx; one rqio per register-resident pass
    const size_t bytes =
        mats_off + (nops * 32 + nfops * (sizeof(rq_layout) / sizeof(cx)) +
                    items.size() * (sizeof(rqio) / sizeof(cx))) *
                       sizeof(cx);
    if (dry && bytes > prog_cap) {
      dry_prog.resize(bytes);
      prog_host = dry_prog.data();
      prog_cap = bytes;
    }
    if (bytes > prog_cap) {
      QDC_TRY(sync_all());
      for (auto& d : devs) {
        QDC_TRY(d->ctx.use());
        if (d->prog_dev) QDC_HIP(hipFree(d->prog_dev));
        d->prog_dev = nullptr;
        QDC_HIP(hipMalloc(&d->prog_dev, bytes));
      }
      if (prog_host) QDC_HIP(hipHostFree(prog_host));
      prog_host = nullptr;
      QDC_HIP(hipHostMalloc(&prog_host, bytes));
      prog_cap = bytes;
    }
    fop* fops = reinterpret_cast<fop*>(prog_host);
    cx* mats = reinterpret_cast<cx*>(prog_host + mats_off);
    size_t fo = 0, mo = 0;
    uint32_t next_slot = nvar;
    for (size_t ii = 0; ii < items.size(); ++ii) {
      Item& it = items[ii];
      if (it.type != 2) continue;
      it.fop_off = fo * sizeof(fop);
      it.grad_slots.clear();
      it.flops_per_amp = 0;
      const bool two = backward && it.ops[0] >= first_inject;
      it.has_red = false;
      it.writes_f = false;
      std::vector<fop> pf;  // the pass's stage ops in program order
      std::vector<uint64_t> pq;  // their qubits (physical positions)
      std::vector<uint32_t> pc;  // their order classes (qdc_fusion.hpp)
      std::vector<int> pslot;    // their reduction slot (Gamma stages), else -1
      pf.reserve(it.stages.size());
      const FusionPlanner PL = planner();
      for (const auto& st : it.stages) {
        uint64_t q = 0;
        uint32_t c = 0;
        for (uint32_t pi : st) {
          q |= (1ull << plan[pi].pos2) | (1ull << plan[pi].pos1);
          c |= PL.op_class(plan[pi], backward);
        }
        pq.push_back(q);
        pc.push_back(c);
      }
      auto local_bit = [&](uint32_t p) -> uint32_t {
        if (p < (uint32_t)LV + it.lc) return p;
        for (uint32_t r = 0; r < it.h; ++r)
          if (it.hb[r] == p - LV) return LV + it.lc + r;
        return 0xffffffffu;  // unreachable: tile_config covered every bit
      };
      if (rec_mats) (*rec_mats)[ii].clear();
      for (size_t sj = 0; sj < it.stages.size(); ++sj) {
        const auto& st = it.stages[sj];
        if (rec_mats && is_meas(plan[st[0]])) (*rec_mats)[ii].push_back(smat_identity(2));
        if (is_meas(plan[st[0]])) {  // density (forward) or cotangent injection (backward)
          const qdc_plan_op& op = plan[st[0]];
          const Instr& in = ins[op.instr];
          const bool q1 = is_q1_density(in.kind);
          const int R = q1 ? 2 : 4;
          pf.emplace_back();
          pslot.push_back(-1);
          fop& F = pf.back();
          F.t1 = local_bit(q1 ? op.pos2 : op.pos1);
          F.t2 = local_bit(op.pos2);
          F.mat = (uint32_t)mo;
          for (int i = 0; i < 2 * R * R; ++i) mats[mo + i] = cx{0, 0};
          if (backward) {  // b += (G^T on pos) (2 conj f), G = conj of the JAX cotangent
            F.kind = q1 ? FK_INJ1 : FK_INJ2;
            const qdc_complex* gd = dg->at(gidx[op.instr]);
            if (q1) {
              const mat<2> m = transpose<2>(to_mat<2>(gd));
              for (int i = 0; i < 4; ++i) mats[mo + i] = m.a[i];
            } else {
              const mat<4> m = transpose<4>(to_mat<4>(gd));
              for (int i = 0; i < 16; ++i) mats[mo + i] = m.a[i];
            }
            it.flops_per_amp += 8.0 * (q1 ? 2.0 : 4.0);
          } else {
            F.kind = q1 ? FK_DENS1 : FK_DENS2;
            it.grad_slots.push_back(out_idx[op.instr]);
            it.has_red = true;
            it.flops_per_amp += 8.0 * (q1 ? 2.0 : 4.0);
          }
          mo += 2 * R * R;
          continue;
        }
        // stage qubits (physical positions), lo < hi
        uint64_t qm = 0;
        bool all_diag = true, any_grad = false;
        for (uint32_t pi : st) {
          qm |= (1ull << plan[pi].pos2) | (1ull << plan[pi].pos1);
          all_diag = all_diag && is_diag(ins[plan[pi].instr].kind);
          any_grad = any_grad || (two && is_var(ins[plan[pi].instr].kind));
        }
        const uint32_t lo = (uint32_t)__builtin_ctzll(qm);
        const uint32_t hi = 63u - (uint32_t)__builtin_clzll(qm);
        const int R = lo == hi ? 2 : 4;
        SMat A = smat_identity(R);
        SMatD B = smat_identity<double>(R);
        StagePost post;
        post.R = R;
        post.diag_only = all_diag;
        for (uint32_t pi : st) {
          const qdc_plan_op& op = plan[pi];
          const Instr& in = ins[op.instr];
          const qdc_complex* g4 = is_const(in.kind) ? cg.at(gidx[op.instr]) : vg.at(gidx[op.instr]);
          const bool dg = is_diag(in.kind);
          int role;
          if (R == 2)
            role = ROLE_Q1_ONLY;
          else if (is_q1_gate(in.kind))
            role = op.pos2 == lo ? ROLE_Q1_LO : ROLE_Q1_HI;
          else
            role = op.pos2 == hi ? ROLE_Q2 : ROLE_Q2_SWAP;
          // the applied matrix a (forward: U; uncompute: U^dagger / U^-1 / conj diagonal) and
          // the pull-back b = U^T (diagonal: d), each in the gate's own basis
          cd ga[16];
          cdd gb[16];
          if (dg) {
            const diag4 d = to_diag(g4);
            const diag4 a = backward ? conj_diag(d) : d;
            for (int i = 0; i < 4; ++i) {
              ga[i] = cd(a.a[i].x, a.a[i].y);
              gb[i] = cdd(d.a[i].x, d.a[i].y);
            }
          } else if (is_q1_gate(in.kind)) {
            const mat<2> u = to_mat<2>(g4);
            mat<2> a = u;
            if (backward) {
              if (is_nonu(in.kind))
                QDC_TRY(inverse<2>(u, a));
              else
                a = conj_transpose<2>(u);
            }
            const mat<2> bt = transpose<2>(u);
            for (int i = 0; i < 4; ++i) {
              ga[i] = cd(a.a[i].x, a.a[i].y);
              gb[i] = cdd(bt.a[i].x, bt.a[i].y);
            }
          } else {
            const mat<4> u = to_mat<4>(g4);
            mat<4> a = u;
            if (backward) {
              if (is_nonu(in.kind))
                QDC_TRY(inverse<4>(u, a));
              else
                a = conj_transpose<4>(u);
            }
            const mat<4> bt = transpose<4>(u);
            for (int i = 0; i < 16; ++i) {
              ga[i] = cd(a.a[i].x, a.a[i].y);
              gb[i] = cdd(bt.a[i].x, bt.a[i].y);
            }
          }
          const SMat Ea = stage_embed(ga, dg, role, R);
          const SMatD Eb = stage_embed(gb, dg, role, R);
          const SMat Anew = smat_mul(Ea, A);
          if (two && is_var(in.kind))
            post.gates.push_back(StageGate{var_idx[op.instr], dg, role, B, smat_double(smat_transpose(Anew))});
          A = Anew;
          B = smat_mul(Eb, B);
        }
        if (rec_mats) (*rec_mats)[ii].push_back(A);  // the forward's matrix, its own frame
        // a mirrored backward stage uncomputes with exactly the adjoint of the forward's matrix
        // (same rounding; the forward frame's two qubits may have swapped order under the
        // forward pass's permutation)
        SMat Aup = A;
        bool from_fwd = false;
        if (backward && !it.mirror_of.empty()) {
          bool nonu = false;
          for (uint32_t pi : st) nonu = nonu || is_nonu(ins[plan[pi].instr].kind);
          const auto& mo_ = it.mirror_of[sj];
          if (!nonu && mo_.first < mrec.stage_mats.size() && mo_.second < mrec.stage_mats[mo_.first].size()) {
            const SMat& Pf = mrec.stage_mats[mo_.first][mo_.second];
            if (Pf.R == R) {
              // forward lo / hi positions vs this stage's: swapped when the forward's lower
              // qubit now sits above the other
              uint32_t flo = 64, fhi = 0;
              for (uint32_t fi : mrec.items[mo_.first].stages[mo_.second]) {
                const qdc_plan_op& fo = mrec.plan[fi];
                flo = std::min({flo, fo.pos2, fo.pos1});
                fhi = std::max({fhi, fo.pos2, fo.pos1});
              }
              const auto& fsw = mrec.items[mo_.first].swaps;
              auto sig = [&](uint32_t p) {
                for (const auto& sw : fsw) {
                  if (p == sw.first) p = sw.second;
                  else if (p == sw.second) p = sw.first;
                }
                return p;
              };
              const bool swapped = R == 4 && sig(flo) > sig(fhi);
              SMat At = Pf;
              for (int pp = 0; pp < R; ++pp)
                for (int qq = 0; qq < R; ++qq) {
                  const int sp = swapped ? swap_bits4(pp) : pp, sq = swapped ? swap_bits4(qq) : qq;
                  At.a[pp * R + qq] = std::conj(Pf.a[sq * R + sp]);
                }
              Aup = At;
              from_fwd = true;
            }
          }
        }
        if (tracing) {  // (physical positions; trace_logical maps them to logical qubits)
          TraceOp t{backward ? 1u : 0u, (uint32_t)ii, hi, lo, (uint32_t)R, all_diag ? 1u : 0u,
                    from_fwd ? 1u : 0u, 0u, {}};
          for (int i = 0; i < R * R; ++i) {
            const bool keep = !all_diag || i % (R + 1) == 0;
            t.m[i].re = keep ? (qdc_real)(real)Aup.a[i].real() : 0;
            t.m[i].im = keep ? (qdc_real)(real)Aup.a[i].imag() : 0;
          }
          trace.push_back(t);
        }
        pf.emplace_back();
        pslot.push_back(-1);
        fop& F = pf.back();
        F.t1 = local_bit(lo);
        F.t2 = local_bit(hi);
        F.mat = (uint32_t)mo;
        const uint32_t kind = all_diag ? FK_DIAG : (R == 2 ? FK_Q1 : FK_Q2);
        F.kind = kind | (any_grad ? FOP_GAMMA : 0u);
        it.writes_f = true;
        const int n = all_diag ? 4 : R * R;
        for (int i = 0; i < n; ++i) {
          const cd va = all_diag ? Aup.a[i * 4 + i] : Aup.a[i];
          const cdd vb = all_diag ? B.a[i * 4 + i] : B.a[i];
          mats[mo + i] = cx{(real)va.real(), (real)va.imag()};
          mats[mo + n + i] = cx{(real)vb.real(), (real)vb.imag()};
        }
        mo += 2 * n;
        // complex MACs per amplitude: 1 (diagonal), 2 (one qubit), 4 (two qubits) per matrix
        // applied (A; B too when two-state) and per Gamma accumulated; 8 real FLOPs each
        const double cmac = all_diag ? 1.0 : (R == 2 ? 2.0 : 4.0);
        it.flops_per_amp += 8.0 * cmac * ((two ? 2.0 : 1.0) + (any_grad ? 1.0 : 0.0));
        if (any_grad) {
          post.slot = next_slot++;
          it.grad_slots.push_back(post.slot);
          pslot.back() = (int)post.slot;
          it.has_red = true;
          stage_post.push_back(std::move(post));
        }
      }
      // register-resident pass: f32, gate stages only (no densities / injections)
      bool rq = use_rq && (sizeof(real) == 4 || rq64) && it.writes_f;
      for (const fop& F : pf) rq = rq && (F.kind & 7u) <= FK_DIAG;
      it.rq = rq;
      if (!it.swaps.empty() && !rq)
        return fail("internal: a permuting fused pass is not register-resident");
      it.tbits = (uint32_t)LV + it.lc + it.h;
      // the kernels index their per-wave accumulators by reduction op: a pass with more
      // reduction ops than accumulators is a planner bug, never folded into another slot
      {
        const size_t nred = it.grad_slots.size();
        const size_t cap = rq ? (size_t)FMAX_GRAD_RQ : (size_t)FMAX_GRAD;
        if (nred > cap)
          return fail("internal: a fused pass has %zu reduction ops, the kernel holds %zu", nred,
                      cap);
      }
      if (!rq) {
        for (const fop& F : pf) fops[fo++] = F;
        it.nstage = (uint32_t)pf.size();
        bool d1 = dens1_kernel && !two && !it.writes_f && !pf.empty() && pf.size() <= (size_t)DENS1_MAX;
        for (const fop& F : pf) d1 = d1 && (F.kind & 7u) == FK_DENS1;
        it.dens1 = d1;
        continue;
      }
      auto put_layout = [&](const RqLayout& L) {
        const rq_layout d = rq_descriptor(L, it.tbits);
        const uint32_t off = (uint32_t)mo;
        std::memcpy(&mats[mo], &d, sizeof d);
        mo += sizeof(rq_layout) / sizeof(cx);
        return off;
      };
      std::vector<RqStage> rs;
      for (size_t k = 0; k < pf.size(); ++k) {
        RqStage r{pf[k].kind & 7u, pf[k].t1, pf[k].t2, 0};
        for (size_t i = 0; i < k; ++i)
          if ((pq[i] & pq[k]) || (FusionPlanner::conflicts_of(pc[i]) & pc[k]) ||
              (FusionPlanner::conflicts_of(pc[k]) & pc[i]))
            r.deps |= 1ull << i;
        rs.push_back(r);
      }
      // a permuting pass: tile bit t's value is stored where tile bit dest[t] sits
      uint32_t dest[32], src[4] = {0, 1, 2, 3};
      const bool perm = !it.swaps.empty();
      if (perm) {
        for (uint32_t t = 0; t < it.tbits; ++t) {
          uint32_t p = t < (uint32_t)LV + it.lc ? t : (uint32_t)LV + it.hb[t - LV - it.lc];
          for (const auto& sw : it.swaps) {
            if (p == sw.first) p = sw.second;
            else if (p == sw.second) p = sw.first;
          }
          dest[t] = local_bit(p);
          if (dest[t] < 4) src[dest[t]] = t;
        }
      }
      // five register slots on the one-wave two-state f32 kernel (k_rw<.., S5>)
      const bool s5_two = two && rq5();
      const bool s5_one = !two && ((rq_slots5 && rw1() && it.tbits == 11) ||  // k_rw W = 1
                                   (rq_fwd5 && it.tbits == 12));  // k_rw W = 2, prefetching
      const uint32_t ns = (sizeof(real) == 4 && (s5_two || s5_one)) ? 5u : 4u;
      it.s5 = ns == 5;
      const bool keep = spec_half && ns == 5 && it.tbits == 11 && sizeof(real) == 4;
      const RqPlan& P = rq_plan_cached(rs, it.tbits, perm ? src : nullptr, rq_maxcl != 0, ns, keep);
      it.l0 = put_layout(P.load);
      {  // rqio after the load descriptor
        rqio io{};
        rq_hbm(P.load, it.tbits, it.lc, it.hb, io.gv_ld, io.offi_ld);
        rq_hbm(P.store, it.tbits, it.lc, it.hb, io.gv_st, io.offi_st, perm ? dest : nullptr);
        // gapped offsets (interleaved pair): the kernel gaps only the tile base, and the gap
        // is linear over the disjoint bit sets of base, thread and register offsets
        for (uint64_t* a : {io.gv_ld, io.gv_st})
          for (int k = 0; k < 8; ++k) a[k] += a[k] & gm;
        for (uint64_t* a : {io.offi_ld, io.offi_st})
          for (int k = 0; k < RQ_R; ++k) a[k] += a[k] & gm;
        std::memcpy(&mats[mo], &io, sizeof io);
        mo += sizeof(rqio) / sizeof(cx);
      }
      uint32_t n = 0;
      it.grad_slots.clear();  // the kernel reduces Gamma stages in execution order
      // the kernels launch_rq runs: f32 two-state five-slot k_rw, one-state prefetching k_rq on
      // 2^12 tiles; f64 two-state k_rw on 2^10 tiles, one-state on 2^10 / 2^11
      const bool f32 = sizeof(real) == 4;
      const bool spec1 = spec_on() && spec_fwd && !two &&
                         (f32 ? ((!it.s5 && it.tbits == 12 && rq_prefetch && !(rq_wave & 2)) ||
                                 (it.s5 && it.tbits == 11 && rw1()))
                              : (it.tbits == 10 || it.tbits == 11));
      const bool spec = spec1 || (spec_on() && two && (f32 ? (it.s5 && rq5()) : it.tbits == 10));
      std::vector<SpecStep> sst;
      RqLayout lcur = P.load;
      it.spec = nullptr;
      for (const RqStep& step : P.steps) {
        if (!step.relayout && pslot[step.stage] >= 0)
          it.grad_slots.push_back((uint32_t)pslot[step.stage]);
        fop F{};
        if (step.relayout) {
          F.kind = FK_RELAYOUT;
          F.mat = put_layout(step.L);
          if (spec) sst.push_back(SpecStep{true, lcur, step.L, F});
          lcur = step.L;
        } else {
          F = pf[step.stage];
          F.t1 = step.cs;
          F.t2 = 0;
          // two-qubit / diagonal stages run with the lower slot first (half the kernel's
          // cases): exchange t1 and t2 by permuting the matrices' index bits, and the
          // stage's Gamma back on the host
          const uint32_t kd = F.kind & 7u;
          if ((kd == FK_Q2 || kd == FK_DIAG) && (step.cs >> 3) > (step.cs & 7u)) {
            F.t1 = (step.cs & 7u) * 8u + (step.cs >> 3);
            const int nm = kd == FK_DIAG ? 4 : 16;
            for (int h = 0; h < 2; ++h) {  // A, then B
              cx* m = &mats[F.mat + (size_t)h * nm];
              cx t[16];
              for (int i = 0; i < nm; ++i) t[i] = m[i];
              for (int i = 0; i < nm; ++i)
                m[i] = kd == FK_DIAG ? t[swap_bits4(i)]
                                     : t[swap_bits4(i >> 2) * 4 + swap_bits4(i & 3)];
            }
            if (pslot[step.stage] >= 0)
              for (StagePost& sp : stage_post)
                if (sp.slot == (uint32_t)pslot[step.stage]) sp.swapped = true;
          }
        }
        if (spec && !step.relayout) sst.push_back(SpecStep{false, lcur, lcur, F});
        fops[fo++] = F;
        ++n;
      }
      it.nstage = n;
      if (spec) {
        // the source is generated once per distinct program (per process): the key is
        // everything it depends on, the layouts, stage kinds, slot cases and Γ flags
        const bool pf1 = spec1 && it.s5 && rw1_prefetch();
        const bool half1 = it.s5 && it.tbits == 11 && !pf1 && spec_half && !spec_imm() &&
                           sizeof(real) == 4 && spec_half_ok(sst);
        std::vector<uint32_t> key = {spec1 ? 1u : 2u, it.tbits, spec_imm() ? 1u : 0u,
                                     (pf1 ? 1u : 0u) | (half1 ? 2u : 0u)};
        auto put_layout_key = [&](const RqLayout& L) {
          key.push_back(L.ns | (L.tfix ? 0x100u : 0u));
          for (uint32_t q = 0; q < RQ_SLOTS_MAX; ++q) key.push_back(L.slot[q]);
          for (int q = 0; q < 3; ++q) key.push_back(L.tfirst[q]);
        };
        put_layout_key(P.load);
        for (const SpecStep& ss : sst) {
          if (ss.relayout) {
            key.push_back(0xffffffffu);
            put_layout_key(ss.Ln);
          } else {
            key.push_back(ss.F.kind);
            key.push_back(ss.F.t1);
          }
        }
        auto hit = spec_cache.find(key);
        if (hit == spec_cache.end()) {
          const SpecKind K = spec1 ? spec_kind_one(it.tbits, pf1, half1) : spec_kind_two(half1);
          const std::string body = spec_program_source(sst, it.tbits, K);
          SpecEntry e;
          e.name = spec_kernel_name(body, K);
          e.src = spec_kernel_source(e.name, body, K);
          hit = spec_cache.emplace(std::move(key), std::move(e)).first;
        }
        it.spec = &hit->second;
      }
      if (rq_stats) fprintf(stderr, "rq pass: %zu stages, %u ops (T=%u lc=%u)\n", pf.size(), n, it.tbits, it.lc);
      if (rq_stats >= 2) {  // the pass's stages for offline planner studies (tools/)
        fprintf(stderr, "rq stages %s T=%u perm=%d:", two ? "two" : "one", it.tbits, perm ? 1 : 0);
        for (const RqStage& r : rs)
          fprintf(stderr, " %u,%u,%u,%llx", r.kind, r.t1, r.t2, (unsigned long long)r.deps);
        fprintf(stderr, "\n");
      }
    }
    if (dry) {  // the kernels this call would compile / load
      for (Item& it : items)
        if (it.spec && std::find(dry_specs.begin(), dry_specs.end(), it.spec) == dry_specs.end())
          dry_specs.push_back(it.spec);
      return nullptr;
    }
    for (auto& d : devs) {  // prog_host is not rewritten before the call's final sync
      QDC_TRY(d->ctx.use());
      QDC_HIP(hipMemcpyAsync(d->prog_dev, prog_host, mats_off + mo * sizeof(cx),
                             hipMemcpyHostToDevice, d->ctx.stream));
    }
    QDC_TRY(spec_load(items));
    return nullptr;
  }
  // specialized passes: circuits of >= spec_min_qubits local qubits (every shard runs the same
  // program; the kernels are loaded on each shard's device)
  bool spec_on() const { return spec_mode > 0 && (spec_mode >= 2 || nl >= spec_min_qubits); }
  // compile / load the kernels of this program's specialized passes (more distinct ones than
  // spec_max — deep random circuits would compile for minutes — go to the background compiler)
  const char* spec_load(std::vector<Item>& items) {
    if (items.empty()) return nullptr;
    size_t distinct = 0;
    ++spec_epoch;
    for (Item& it : items)
      if (it.spec && it.spec->epoch != spec_epoch) {
        it.spec->epoch = spec_epoch;
        ++distinct;
      }
    if (distinct == 0) return nullptr;
    const bool async = distinct > spec_max;
    if (async && !spec_async) {  // every pass of this call interpreted
      for (Item& it : items) it.spec = nullptr;
      return nullptr;
    }
    std::vector<int> devs;
    for (auto& s : sh)
      if (std::find(devs.begin(), devs.end(), s.c().device) == devs.end()) devs.push_back(s.c().device);
    for (size_t di = 0; di < devs.size(); ++di) {
      const int dev = devs[di];
      std::vector<SpecEntry*> todo;  // distinct kernels not loaded on dev yet
      ++spec_epoch;
      for (Item& it : items)
        if (it.spec && it.spec->epoch != spec_epoch) {
          it.spec->epoch = spec_epoch;
          if (!it.spec->fn.count(dev)) todo.push_back(it.spec);
        }
      if (todo.empty()) continue;
      std::vector<std::string> names, srcs;
      for (const SpecEntry* e : todo) {
        names.push_back(e->name);
        srcs.push_back(e->src);
      }
      for (auto& s : sh)
        if (s.c().device == dev) {
          QDC_TRY(s.c().use());
          break;
        }
      std::vector<hipFunction_t> fns;
      if (async)  // (what is compiled loads now, the rest compiles in the background)
        SpecJit::get().ensure_async(dev, names, srcs, fns);
      else
        SpecJit::get().ensure(dev, names, srcs, fns);
      for (size_t k = 0; k < todo.size(); ++k)
        if (fns[k]) todo[k]->fn[dev] = fns[k];
    }
    return nullptr;
  }
  // the pass's specialized kernel on a device, or none (the interpreted kernel runs)
  static hipFunction_t spec_fn_on(const Item& it, int dev) {
    if (!it.spec) return nullptr;
    auto f = it.spec->fn.find(dev);
    return f == it.spec->fn.end() ? nullptr : f->second;
  }
  // Run one fused group on every shard.  grads != nullptr: two-state reverse program whose
  // gradient gates write partials for gradient buffer rows var_idx[...].
  template <bool TWO, bool HASRED, bool WF, int NT>
  static auto fused_kernel() {
    constexpr int TB = TWO ? (int)TILE_CHUNKS_2 : (int)TILE_CHUNKS_1;
    return k_fused<TWO, TB, HASRED, WF, NT>;
  }
  template <bool TWO, bool HASRED, bool WF>
  const char* launch_fused(Ctx& ctx, const char* name, double bytes, const fgeo& fg, chunk* f,
                           chunk* b, const fop* fops, const cx* mats, cx* partials,
                           uint64_t stride) {
    // one-state passes on the smaller tile (QDC_TILE1_CHUNKS = TILE_CHUNKS_2): the LDS kernel
    // of that tile size (a k_fused tile is always TB chunks)
    if constexpr (!TWO) {
      if ((1ull << (fg.lc + fg.h)) == TILE_CHUNKS_2)
        return launch_fused_tb<TWO, HASRED, WF, (int)TILE_CHUNKS_2>(ctx, name, bytes, fg, f, b, fops,
                                                                    mats, partials, stride);
    }
    constexpr int TB = TWO ? (int)TILE_CHUNKS_2 : (int)TILE_CHUNKS_1;
    return launch_fused_tb<TWO, HASRED, WF, TB>(ctx, name, bytes, fg, f, b, fops, mats, partials, stride);
  }
  template <bool TWO, bool HASRED, bool WF, int TB>
  const char* launch_fused_tb(Ctx& ctx, const char* name, double bytes, const fgeo& fg, chunk* f,
                              chunk* b, const fop* fops, const cx* mats, cx* partials,
                              uint64_t stride) {
    if ((1ull << (fg.lc + fg.h)) != (uint64_t)TB)
      return fail("internal: a %llu-chunk fused tile on the %d-chunk LDS kernel",
                  (unsigned long long)(1ull << (fg.lc + fg.h)), TB);
    // 256 threads per tile (measured: 128 threads with twice the quartets per thread and
    // occupancy 2 was 2-4 % slower)
    constexpr int NT = 256;
    auto kern = k_fused<TWO, TB, HASRED, WF, NT>;
    uint32_t grid = 0;
    QDC_TRY(fused_grid(fg, (const void*)kern, NT, grid));
    fgeo g = fg;
    uint64_t tpb = 1;
    while (tpb * grid < g.ntiles) tpb <<= 1;
    g.tpb = (uint32_t)tpb;
    grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
    if (g.ngrad > 0 && grid > NBMAX) return fail("fused reduction grid %u exceeds %u", grid, NBMAX);
    last_fused_grid = grid;
    last_fused_ndyn = 0;
    return ctx.launch_block(name, bytes, kern, grid, (uint32_t)NT, f, b, fops, mats, g, partials,
                            stride);
  }
  // a density-only pass (k_dens1): the tile of the one-state LDS kernel of its size
  const char* launch_dens1(Ctx& ctx, const char* name, double bytes, const fgeo& fg, chunk* f,
                           const fop* fops, cx* partials, uint64_t stride) {
    if ((1ull << (fg.lc + fg.h)) == TILE_CHUNKS_2)
      return launch_dens1_tb<(int)TILE_CHUNKS_2>(ctx, name, bytes, fg, f, fops, partials, stride);
    return launch_dens1_tb<(int)TILE_CHUNKS_1>(ctx, name, bytes, fg, f, fops, partials, stride);
  }
  template <int TB>
  const char* launch_dens1_tb(Ctx& ctx, const char* name, double bytes, const fgeo& fg, chunk* f,
                              const fop* fops, cx* partials, uint64_t stride) {
    if ((1ull << (fg.lc + fg.h)) != (uint64_t)TB)
      return fail("internal: a %llu-chunk density tile on the %d-chunk kernel",
                  (unsigned long long)(1ull << (fg.lc + fg.h)), TB);
    if (fg.nops == 0 || fg.nops > (uint32_t)DENS1_MAX || fg.ngrad != fg.nops)
      return fail("internal: a density pass of %u ops, %u reductions", fg.nops, fg.ngrad);
    constexpr int NT = 256;
    auto kern = k_dens1<TB, NT>;
    uint32_t grid = 0;
    QDC_TRY(fused_grid(fg, (const void*)kern, NT, grid));
    fgeo g = fg;
    uint64_t tpb = 1;
    while (tpb * grid < g.ntiles) tpb <<= 1;
    g.tpb = (uint32_t)tpb;
    grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
    if (grid > NBMAX) return fail("density reduction grid %u exceeds %u", grid, NBMAX);
    last_fused_grid = grid;
    last_fused_ndyn = 0;
    return ctx.launch_block(name, bytes, kern, grid, (uint32_t)NT, (const chunk*)f, fops, g,
                            partials, stride);
  }
  // register-resident pass (qdc_rq.hpp): threads per tile = tile amplitudes / RQ_R
  const char* launch_rq(Ctx& ctx, const char* name, double bytes, const fgeo& fg, bool two,
                        uint32_t tbits, uint32_t l0, chunk* f, chunk* b, const fop* fops,
                        const cx* mats, cx* partials, uint64_t stride, bool s5,
                        hipFunction_t spec = nullptr) {
#ifndef QDC_F64
    const uint32_t nt = (1u << tbits) / (uint32_t)RQ_R;
    if (!two && s5 && nt == 256) {  // two waves per 2^12 tile, five slots, prefetching
      const void* kw = (const void*)k_rw<false, 2, true, 2, true>;
      uint32_t grid = 0;
      QDC_TRY(fused_grid(fg, kw, 128, grid));
      fgeo g = fg;
      if (!(g.ngrad == 0 && grid >= 8 && g.ntiles >= 4ull * grid && ctx.plan_dyn(g, grid))) {
        uint64_t tpb = 1;
        while (tpb * grid < g.ntiles) tpb <<= 1;
        g.tpb = (uint32_t)tpb;
        grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
      }
      last_fused_grid = grid;
      last_fused_ndyn = 0;
      return ctx.launch_block(name, bytes, k_rw<false, 2, true, 2, true>, grid, 128u, f, b, fops,
                              mats, g, l0, partials, stride);
    }
    if (!two && s5 && nt == 128 && rw1_prefetch()) {  // one wave per 2^11 tile, prefetching
      const void* kw = (const void*)k_rw<false, 2, true, 1, true>;
      uint32_t grid = 0;
      QDC_TRY(fused_grid(fg, kw, 64, grid));
      fgeo g = fg;
      if (!(g.ngrad == 0 && grid >= 8 && g.ntiles >= 4ull * grid && ctx.plan_dyn(g, grid))) {
        uint64_t tpb = 1;
        while (tpb * grid < g.ntiles) tpb <<= 1;
        g.tpb = (uint32_t)tpb;
        grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
      }
      last_fused_grid = grid;
      last_fused_ndyn = 0;
      if (spec)
        return ctx.launch_module(name, bytes, spec, grid, 64u, f, b, fops, mats, g, l0, partials, stride);
      return ctx.launch_block(name, bytes, k_rw<false, 2, true, 1, true>, grid, 64u, f, b, fops,
                              mats, g, l0, partials, stride);
    }
    if ((two ? (rq_wave & 1) : ((rq_wave & 2) || (rw1() && nt == 128))) &&
        (nt == 128 || (nt == 256 && !two))) {
      // k_rw: lane l of a tile's W waves runs k_rq's threads l + 64 W e (e < 2)
      const bool pfw = two && (rq_wave & 4);
      const uint32_t bs = (!two && nt == 256) ? 128u : 64u;
      if (s5 && !((two && !pfw) || (!two && nt == 128)))
        return fail("internal: a five-slot pass without its kernel");
      const void* kw = two ? (pfw  ? (const void*)k_rw<true, 2, true, 1>
                              : s5 ? (const void*)k_rw<true, 2, false, 1, true>
                                   : (const void*)k_rw<true, 2, false, 1>)
                           : nt == 128 ? (s5 ? (const void*)k_rw<false, 2, false, 1, true>
                                             : (const void*)k_rw<false, 2, false, 1>)
                                       : (const void*)k_rw<false, 2, false, 2>;
      uint32_t grid = 0;
      QDC_TRY(fused_grid(fg, kw, (int)bs, grid));
      if (nt == 128 && s5 && spec && !(two && pfw)) QDC_TRY(fused_grid_fn(spec, (int)bs, grid));
      fgeo g = fg;
      // one wave per block: static shares + a dynamic tail
      if (!(bs == 64 && !pfw && grid >= 8 && g.ntiles >= 4ull * grid && ctx.plan_dyn(g, grid))) {
        uint64_t tpb = 1;
        while (tpb * grid < g.ntiles) tpb <<= 1;
        g.tpb = (uint32_t)tpb;
        grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
      }
      if (g.ngrad > 0 && grid > NBMAX) return fail("fused reduction grid %u exceeds %u", grid, NBMAX);
      last_fused_grid = grid;
      last_fused_ndyn = g.ndyn ? ctx.last_ndyn : 0u;
      if (two && pfw)
        return ctx.launch_block(name, bytes, k_rw<true, 2, true, 1>, grid, bs, f, b, fops, mats, g,
                                l0, partials, stride);
      if (two && s5 && spec)  // the pass's straight-line kernel (same resources and grid)
        return ctx.launch_module(name, bytes, spec, grid, bs, f, b, fops, mats, g, l0, partials,
                                 stride);
      if (two && s5)
        return ctx.launch_block(name, bytes, k_rw<true, 2, false, 1, true>, grid, bs, f, b, fops,
                                mats, g, l0, partials, stride);
      if (two)
        return ctx.launch_block(name, bytes, k_rw<true, 2, false, 1>, grid, bs, f, b, fops, mats, g,
                                l0, partials, stride);
      if (nt == 128 && s5 && spec)  // one-wave one-state pass, specialized
        return ctx.launch_module(name, bytes, spec, grid, bs, f, b, fops, mats, g, l0, partials,
                                 stride);
      if (nt == 128 && s5)
        return ctx.launch_block(name, bytes, k_rw<false, 2, false, 1, true>, grid, bs, f, b, fops,
                                mats, g, l0, partials, stride);
      if (nt == 128)
        return ctx.launch_block(name, bytes, k_rw<false, 2, false, 1>, grid, bs, f, b, fops, mats, g,
                                l0, partials, stride);
      return ctx.launch_block(name, bytes, k_rw<false, 2, false, 2>, grid, bs, f, b, fops, mats, g,
                              l0, partials, stride);
    }
    const void* kern = nullptr;
    // the next tile's loads are in flight while this tile's stages run (2 waves/SIMD)
    const bool pf = two ? rq_prefetch2 != 0 : rq_prefetch != 0;
    if (two && nt == 128) kern = pf ? (const void*)k_rq<true, 128, true> : (const void*)k_rq<true, 128, false>;
    else if (!two && nt == 128) kern = pf ? (const void*)k_rq<false, 128, true> : (const void*)k_rq<false, 128, false>;
    else if (!two && nt == 256) kern = pf ? (const void*)k_rq<false, 256, true> : (const void*)k_rq<false, 256, false>;
    else return fail("no register-resident kernel for a %u-amplitude %s tile", 1u << tbits,
                     two ? "two-state" : "one-state");
    uint32_t grid = 0;
    QDC_TRY(fused_grid(fg, kern, (int)nt, grid));
    fgeo g = fg;
    // one-state prefetching passes: static shares + a dynamic tail (no reductions here)
    if (!(!two && pf && g.ngrad == 0 && grid >= 8 && g.ntiles >= 4ull * grid &&
          ctx.plan_dyn(g, grid))) {
      uint64_t tpb = 1;
      while (tpb * grid < g.ntiles) tpb <<= 1;
      g.tpb = (uint32_t)tpb;
      grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
    }
    if (g.ngrad > 0 && grid > NBMAX) return fail("fused reduction grid %u exceeds %u", grid, NBMAX);
    last_fused_grid = grid;
    last_fused_ndyn = 0;
    if (!two && nt == 256 && pf && spec)  // the pass's straight-line kernel (same resources and grid)
      return ctx.launch_module(name, bytes, spec, grid, nt, f, b, fops, mats, g, l0, partials, stride);
#define QDC_RQ_LAUNCH(T, N, P)                                                            \
  if (two == T && nt == N && pf == P)                                                     \
    return ctx.launch_block(name, bytes, k_rq<T, N, P>, grid, nt, f, b, fops, mats, g, l0, \
                            partials, stride);
    QDC_RQ_LAUNCH(true, 128, false)
    QDC_RQ_LAUNCH(true, 128, true)
    QDC_RQ_LAUNCH(false, 128, true)
    QDC_RQ_LAUNCH(false, 128, false)
    QDC_RQ_LAUNCH(false, 256, true)
    QDC_RQ_LAUNCH(false, 256, false)
#undef QDC_RQ_LAUNCH
    return fail("no register-resident kernel launched");
#else
    // f64: 16 amplitudes (4 VGPRs each) per lane and state; two-state 2^10-amplitude tiles on one
    // wave, one-state 2^11 on two
    // (a reverse sweep's passes before the first injection are one-state on 2^10 tiles: one wave)
    const uint32_t nt = (1u << tbits) / (uint32_t)RQ_R;
    if (!(two ? nt == 64 : (nt == 64 || nt == 128)))
      return fail("no register-resident kernel for a %u-amplitude %s tile", 1u << tbits,
                  two ? "two-state" : "one-state");
    const void* kw = two        ? (const void*)k_rw<true, 1, false, 1>
                     : nt == 64 ? (const void*)k_rw<false, 1, false, 1>
                                : (const void*)k_rw<false, 1, false, 2>;
    const uint32_t bs = nt;
    uint32_t grid = 0;
    QDC_TRY(fused_grid(fg, kw, (int)bs, grid));
    fgeo g = fg;
    // one wave per block: static shares + a dynamic tail
    if (!(bs == 64 && grid >= 8 && g.ntiles >= 4ull * grid && ctx.plan_dyn(g, grid))) {
      uint64_t tpb = 1;
      while (tpb * grid < g.ntiles) tpb <<= 1;
      g.tpb = (uint32_t)tpb;
      grid = (uint32_t)((g.ntiles + tpb - 1) / tpb);
    }
    if (g.ngrad > 0 && grid > NBMAX) return fail("fused reduction grid %u exceeds %u", grid, NBMAX);
    last_fused_grid = grid;
    last_fused_ndyn = g.ndyn ? ctx.last_ndyn : 0u;
    if (spec)  // the pass's straight-line kernel (same resources and grid)
      return ctx.launch_module(name, bytes, spec, grid, bs, f, b, fops, mats, g, l0, partials, stride);
    if (two)
      return ctx.launch_block(name, bytes, k_rw<true, 1, false, 1>, grid, bs, f, b, fops, mats, g, l0,
                              partials, stride);
    if (nt == 64)
      return ctx.launch_block(name, bytes, k_rw<false, 1, false, 1>, grid, bs, f, b, fops, mats, g, l0,
                              partials, stride);
    return ctx.launch_block(name, bytes, k_rw<false, 1, false, 2>, grid, bs, f, b, fops, mats, g, l0,
                            partials, stride);
#endif
  }
  // one wave of resident blocks (occupancy query, cached per kernel), or QDC_FUSED_BLOCKS
  // (a specialized kernel: its own occupancy, which may differ from the interpreted one's)
  const char* fused_grid_fn(hipFunction_t fn, int nt, uint32_t& grid) {
    if (fused_blocks) {
      grid = fused_blocks;
      return nullptr;
    }
    const void* key = (const void*)fn;
    for (auto& e : fused_resident_cache)
      if (e.first == key) {
        grid = e.second;
        return nullptr;
      }
    int per_cu = 0, dev = 0, cus = 0;
    QDC_HIP(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nt, 0));
    QDC_HIP(hipGetDevice(&dev));
    QDC_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    grid = (uint32_t)std::max(1, std::min(per_cu * cus, (int)NBMAX));
    fused_resident_cache.push_back({key, grid});
    return nullptr;
  }
  const char* fused_grid(const fgeo& fg, const void* kernel, int nt, uint32_t& grid) {
    if (fused_blocks) {
      grid = fused_blocks;
      return nullptr;
    }
    for (auto& e : fused_resident_cache)
      if (e.first == kernel) {
        grid = e.second;
        return nullptr;
      }
    int per_cu = 0, dev = 0, cus = 0;
    QDC_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, nt, 0));
    QDC_HIP(hipGetDevice(&dev));
    QDC_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    grid = (uint32_t)std::max(1, std::min(per_cu * cus, (int)NBMAX));
    fused_resident_cache.push_back({kernel, grid});
    (void)fg;
    return nullptr;
  }

  // Run one fused pass on every shard.  two: fwd and bwd (reverse sweep).  Reductions (Gamma
  // stages, densities) go to slots it.grad_slots of red_base (grads or dens of each shard).
  const char* run_fused(const Item& it, bool two, size_t mats_off, bool red_to_grads) {
    fgeo fg{};
    fg.order = it.rq ? (uint32_t)rq_order : 0u;
    fg.gm = gm;
    fg.lc = it.lc;
    fg.h = it.h;
    for (uint32_t k = 0; k < FMAX_ROWS; ++k) fg.hb[k] = it.hb[k];
    fg.nops = it.nstage;
    fg.ngrad = it.has_red ? (uint32_t)it.grad_slots.size() : 0;
    fg.ntiles = nchunks_of(nl) >> (it.lc + it.h);

    // algorithmic bytes: each state read once, written once if the pass changes it
    const double S = state_bytes(nl);
    const double bytes = two ? (it.writes_f ? 4.0 : 3.0) * S : (it.writes_f ? 2.0 : 1.0) * S;
    const double flops = it.flops_per_amp * (double)((uint64_t)1 << nl);
    // one name per kernel variant (bytes per launch differ: 4S, 3S, 2S, S)
    const char* name = two ? (it.writes_f ? "fused_reverse" : "fused_inject")
                           : (it.writes_f ? "fused_apply" : "fused_density");
    for (auto& s : sh) {
      Ctx& ctx = s.c();
      QDC_TRY(ctx.use());
      const fop* fops = reinterpret_cast<const fop*>(s.d->prog_dev + it.fop_off);
      const cx* mats = reinterpret_cast<const cx*>(s.d->prog_dev + mats_off);
      chunk* f = reinterpret_cast<chunk*>(s.state);
      chunk* b = reinterpret_cast<chunk*>(s.bwd);
      cx* parts = nullptr;
      if (fg.ngrad > 0) {
        cx* base = red_to_grads ? s.grads : s.dens;
        QDC_TRY(ctx.begin_reduction(base, 0));
        if (ctx.pending_dst.size() + fg.ngrad > (size_t)FIN_MAX) QDC_TRY(ctx.flush());
        ctx.pending_base = base;
        ctx.pending_accumulate = 0;
        parts = ctx.slot_ptr();
      }
      const uint64_t stride = (uint64_t)NBMAX * RED;
      ctx.next_flops = flops;
      if (it.rq) {
        QDC_TRY(launch_rq(ctx, name, bytes, fg, two, it.tbits, it.l0, f, b, fops, mats, parts, stride,
                          it.s5, spec_fn_on(it, ctx.device)));
      } else if (two) {
        if (it.writes_f)
          QDC_TRY((launch_fused<true, true, true>(ctx, name, bytes, fg, f, b, fops, mats, parts, stride)));
        else
          QDC_TRY((launch_fused<true, false, false>(ctx, name, bytes, fg, f, b, fops, mats, parts, stride)));
      } else if (it.dens1) {
        QDC_TRY(launch_dens1(ctx, name, bytes, fg, f, fops, parts, stride));
      } else if (!it.has_red) {
        QDC_TRY((launch_fused<false, false, true>(ctx, name, bytes, fg, f, b, fops, mats, parts, stride)));
      } else if (it.writes_f) {
        QDC_TRY((launch_fused<false, true, true>(ctx, name, bytes, fg, f, b, fops, mats, parts, stride)));
      } else {
        QDC_TRY((launch_fused<false, true, false>(ctx, name, bytes, fg, f, b, fops, mats, parts, stride)));
      }
      if (fg.ngrad > 0)
        for (uint32_t slot : it.grad_slots) ctx.commit(slot, last_fused_grid, last_fused_ndyn);
    }
    // a permuting pass stored its tile's qubits at new positions (later ops were planned so)
    for (const auto& sw : it.swaps) layout.swap_phys(sw.first, sw.second);
    return nullptr;
  }

  // --- forward (Circuit::run / Circuit::forward) --------------------------------------------
  const char* apply_gate(Ctx& ctx, const Instr& in, const qdc_complex* g4, cx* s, uint32_t p2,
                         uint32_t p1, bool uncompute) {
    if (is_diag(in.kind)) {
      const diag4 d = to_diag(g4);
      return apply_diag(ctx, s, uncompute ? conj_diag(d) : d, p2, p1, nl,
                        uncompute ? "uncompute_q2_diag" : "apply_q2_diag");
    }
    if (is_q1_gate(in.kind)) {
      const mat<2> u = to_mat<2>(g4);
      mat<2> a = u;
      if (uncompute) {
        if (is_nonu(in.kind))
          QDC_TRY(inverse<2>(u, a));
        else
          a = conj_transpose<2>(u);
      }
      return apply_dense<2>(ctx, s, a, p2, p2, nl, uncompute ? "uncompute_q1" : "apply_q1");
    }
    const mat<4> u = to_mat<4>(g4);
    mat<4> a = u;
    if (uncompute) {
      if (is_nonu(in.kind))
        QDC_TRY(inverse<4>(u, a));
      else
        a = conj_transpose<4>(u);
    }
    return apply_dense<4>(ctx, s, a, p2, p1, nl, uncompute ? "uncompute_q2" : "apply_q2");
  }

  // The trace entries of this call's fused stages (build_program, physical positions) mapped to
  // logical qubits by replaying the call's layout changes (remaps, undone remaps, permuting
  // passes' swaps) from `layout` (the call's start), with the single-gate items' matrices (as
  // apply_gate / reverse_dense apply them) inserted in item order.  Dry runs only.
  const char* trace_logical(const std::vector<Item>& items, const std::vector<qdc_plan_op>& pl,
                            bool backward, const Flat& cg, const Flat& vg,
                            const std::vector<size_t>& gidx) {
    std::vector<TraceOp> fused(trace.begin() + (std::ptrdiff_t)trace_from, trace.end());
    trace.resize(trace_from);
    QubitMap m = layout;
    size_t t = 0;
    for (size_t ii = 0; ii < items.size(); ++ii) {
      const Item& it = items[ii];
      for (; t < fused.size() && fused[t].item == ii; ++t) {
        TraceOp s = fused[t];
        s.q2 = m.logi[s.q2];
        s.q1 = m.logi[s.q1];
        trace.push_back(s);
      }
      if (it.type == 1) {
        const qdc_plan_op& op = pl[it.ops[0]];
        if (it.inv)
          m.unapply(op.victims);
        else
          m.apply(op.victims);
      } else if (it.type == 0) {
        const qdc_plan_op& op = pl[it.ops[0]];
        const Instr& in = ins[op.instr];
        if (is_const(in.kind) || is_var(in.kind)) {
          const qdc_complex* g4 = is_const(in.kind) ? cg.at(gidx[op.instr]) : vg.at(gidx[op.instr]);
          TraceOp s{backward ? 1u : 0u, (uint32_t)ii, m.logi[op.pos2], m.logi[op.pos1], 4u,
                    is_diag(in.kind) ? 1u : 0u, 0u, 1u, {}};
          auto put = [&](const cx* a, int R) {
            s.R = (uint32_t)R;
            for (int i = 0; i < R * R; ++i) s.m[i] = qdc_complex{(qdc_real)a[i].x, (qdc_real)a[i].y};
          };
          if (is_diag(in.kind)) {
            const diag4 d0 = to_diag(g4);
            const diag4 d = backward ? conj_diag(d0) : d0;
            for (int i = 0; i < 4; ++i) s.m[i * 5] = qdc_complex{(qdc_real)d.a[i].x, (qdc_real)d.a[i].y};
          } else if (is_q1_gate(in.kind)) {
            const mat<2> u = to_mat<2>(g4);
            mat<2> a = u;
            if (backward) {
              if (is_nonu(in.kind))
                QDC_TRY(inverse<2>(u, a));
              else
                a = conj_transpose<2>(u);
            }
            s.q1 = s.q2;
            put(a.a, 2);
          } else {
            const mat<4> u = to_mat<4>(g4);
            mat<4> a = u;
            if (backward) {
              if (is_nonu(in.kind))
                QDC_TRY(inverse<4>(u, a));
              else
                a = conj_transpose<4>(u);
            }
            put(a.a, 4);
          }
          trace.push_back(s);
        }
      }
      for (const auto& sw : it.swaps) m.swap_phys(sw.first, sw.second);
    }
    trace_from = trace.size();
    return nullptr;
  }

  const char* dyn_reset_all() {
    for (auto& d : devs) {
      QDC_TRY(d->ctx.use());
      QDC_TRY(d->ctx.dyn_reset());
    }
    return nullptr;
  }
  const char* execute(int mode, const Flat& cg, const Flat& vg, qdc_complex* out) {
    hclock::time_point ht[6];
    ht[0] = hclock::now();
    std::vector<size_t> gidx;
    QDC_TRY(validate_forward(cg, vg, gidx));
    const size_t nout = output_count(mode);
    if (!dry) {
      QDC_TRY(dyn_reset_all());
      QDC_TRY(ensure_out(true, std::max<size_t>(nout, 1) * RED));
    }
    // every pass starts from `initial`, which is always in the identity layout
    layout.identity(n, g);
    for (auto& s : sh) {
      QDC_TRY(s.c().use());
      QDC_TRY(copy_initial(s));
    }
    std::vector<uint32_t> out_idx(ins.size(), 0);
    {
      uint32_t o = 0;
      for (size_t k = 0; k < ins.size(); ++k)
        if (is_diff_density(ins[k].kind) || (mode == QDC_MODE_RUN && is_density(ins[k].kind)))
          out_idx[k] = o++;
    }
    mark_inexact(cg, vg, gidx);
    ht[1] = hclock::now();
    std::vector<qdc_plan_op> pl = plan(mode);
    sched_mirror = mode == QDC_MODE_FORWARD;
    std::vector<Item> items = schedule(pl, false, SIZE_MAX);
    ht[2] = hclock::now();
    size_t mats_off = 0;
    const auto tb0 = std::chrono::steady_clock::now();
    // a mirrored forward records what its backward will undo (forward mode only)
    mrec.valid = false;
    const bool record = mirror_on() && mode == QDC_MODE_FORWARD;
    std::vector<std::vector<SMat>> mats_rec(record ? items.size() : 0);
    rec_mats = record ? &mats_rec : nullptr;
    const char* berr = build_program(items, pl, false, 0, cg, vg, gidx, mats_off, {}, 0, out_idx, nullptr);
    rec_mats = nullptr;
    QDC_TRY(berr);
    ht[3] = hclock::now();
    if (record) {
      mrec.plan = pl;
      mrec.items = items;
      mrec.stage_mats = std::move(mats_rec);
      const size_t nc = cg.size() ? cg.off.back() + cg.len.back() : 0;
      const size_t nv = vg.size() ? vg.off.back() + vg.len.back() : 0;
      mrec.cgates.assign(cg.data, cg.data + nc);
      mrec.vgates.assign(vg.data, vg.data + nv);
      mrec.inexact = inexact;
    }
    if (rq_stats)
      fprintf(stderr, "forward plan+build %.3f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count());
    if (dry) {  // the layout the passes leave (permuting passes' swaps, remaps), no launch
      if (tracing) QDC_TRY(trace_logical(items, pl, false, cg, vg, gidx));
      for (const Item& item : items) {
        for (const auto& sw : item.swaps) layout.swap_phys(sw.first, sw.second);
        if (item.type == 1) layout.apply(pl[item.ops[0]].victims);
      }
      if (record) {
        mrec.end_phys = layout.phys;
        mrec.valid = true;
      }
      return nullptr;
    }
    for (const Item& item : items) {
      if (item.type == 2) {
        QDC_TRY(run_fused(item, false, mats_off, false));
        continue;
      }
      const qdc_plan_op& op = pl[item.ops[0]];
      if (op.type == QDC_PLAN_REMAP) {
        QDC_TRY(remap(op, false));
        continue;
      }
      const Instr& in = ins[op.instr];
      for (auto& s : sh) {
        Ctx& ctx = s.c();
        QDC_TRY(ctx.use());
        if (is_const(in.kind) || is_var(in.kind)) {
          const qdc_complex* g4 = is_const(in.kind) ? cg.at(gidx[op.instr]) : vg.at(gidx[op.instr]);
          QDC_TRY(apply_gate(ctx, in, g4, s.state, op.pos2, op.pos1, false));
        } else if (is_q1_density(in.kind)) {
          QDC_TRY(density<2>(ctx, s.state, op.pos2, op.pos2, nl, s.dens, out_idx[op.instr], 0));
        } else {
          QDC_TRY(density<4>(ctx, s.state, op.pos2, op.pos1, nl, s.dens, out_idx[op.instr], 0));
        }
      }
    }
    ht[4] = hclock::now();
    QDC_TRY(flush_all());
    if (record) {  // (valid once every pass ran; the backward starts from this layout)
      mrec.end_phys = layout.phys;
      mrec.valid = true;
    }
    std::vector<cx*> bufs;
    for (auto& s : sh) bufs.push_back(s.dens);
    QDC_TRY(ex.allreduce(sh, bufs, nout * RED));
    std::vector<int> widths;
    for (auto& in : ins)
      if (is_diff_density(in.kind) || (mode == QDC_MODE_RUN && is_density(in.kind)))
        widths.push_back(is_q1_density(in.kind) ? 4 : 16);
    QDC_TRY(collect(sh[0].dens, widths, out));
    ht[5] = hclock::now();
    host_record(0, ht);
    return nullptr;
  }

  // D2H of `total` (>= widths.size()) result slots into host_out; the first widths.size()
  // are unpacked into `out`.
  const char* collect(const cx* dev, const std::vector<int>& widths, qdc_complex* out,
                      size_t total = 0) {
    const size_t count = widths.size();
    total = std::max(total, count);
    if (total == 0) return sync_all();
    QDC_TRY(ensure_host(total * RED));
    Ctx& c0 = sh[0].c();
    QDC_TRY(c0.use());
    QDC_HIP(hipMemcpyAsync(host_out, dev, sizeof(cx) * total * RED, hipMemcpyDeviceToHost,
                           c0.stream));
    QDC_TRY(sync_all());
    size_t w = 0;
    for (size_t j = 0; j < count; ++j) {
      for (int k = 0; k < widths[j]; ++k) {
        out[w + k].re = host_out[j * RED + k].x;
        out[w + k].im = host_out[j * RED + k].y;
      }
      w += widths[j];
    }
    return nullptr;
  }

  // --- diagonal cotangent injections ----------------------------------------------------------
  // the injection's diagonal (G^T on its qubits has the diagonal of G), or false
  bool diag_cotangent(const qdc_plan_op& op, const Flat& dg, const std::vector<size_t>& gidx) const {
    if (op.type != QDC_PLAN_OP || !is_diff_density(ins[op.instr].kind)) return false;
    const int R = is_q1_density(ins[op.instr].kind) ? 2 : 4;
    if (op.pos2 >= (uint32_t)(4 * DI_GROUPS) || op.pos1 >= (uint32_t)(4 * DI_GROUPS)) return false;
    if (R == 4 && op.pos2 / 4 != op.pos1 / 4) return false;  // both bits in one table group
    const qdc_complex* g = dg.at(gidx[op.instr]);
    for (int p = 0; p < R; ++p)
      for (int q = 0; q < R; ++q)
        if (p != q && (g[p * R + q].re != 0 || g[p * R + q].im != 0)) return false;
    return true;
  }
  // Consecutive items that are injections only, all with diagonal cotangents, become one item of
  // type 3 (their plan ops in order).  Injections only add to bwd from the (unchanged) fwd, so a
  // run of them commutes and sums.
  void merge_diag_injections(std::vector<Item>& items, const std::vector<qdc_plan_op>& pl,
                             const Flat& dg, const std::vector<size_t>& gidx) const {
    auto eligible = [&](const Item& it) {
      if (it.type != 0 && it.type != 2) return false;
      for (uint32_t k : it.ops)
        if (!diag_cotangent(pl[k], dg, gidx)) return false;
      return !it.ops.empty();
    };
    std::vector<Item> out;
    for (Item& it : items) {
      if (eligible(it)) {
        if (!out.empty() && out.back().type == 3) {
          out.back().ops.insert(out.back().ops.end(), it.ops.begin(), it.ops.end());
          continue;
        }
        Item m;
        m.type = 3;
        m.ops = it.ops;
        out.push_back(std::move(m));
        continue;
      }
      out.push_back(std::move(it));
    }
    items = std::move(out);
  }
  // D(i) tables of a type-3 item: T[g * 16 + e] = sum of the diagonal entries that the densities
  // on bits 4g..4g+3 select for the pattern e of those bits (summed in double); returns the
  // number of groups in use
  uint32_t diag_table(const Item& item, const std::vector<qdc_plan_op>& pl, const Flat& dg,
                      const std::vector<size_t>& gidx, diag_tab& T) const {
    cd acc[DI_GROUPS * 16] = {};
    uint32_t ng = 1;
    for (uint32_t k : item.ops) {
      const qdc_plan_op& op = pl[k];
      const bool q1 = is_q1_density(ins[op.instr].kind);
      const int R = q1 ? 2 : 4;
      const qdc_complex* gd = dg.at(gidx[op.instr]);
      const uint32_t grp = op.pos2 / 4;
      ng = std::max(ng, grp + 1);
      for (uint32_t e = 0; e < 16; ++e) {
        const uint32_t b2 = (e >> (op.pos2 % 4)) & 1u, b1 = (e >> (op.pos1 % 4)) & 1u;
        const int r = q1 ? (int)b2 : (int)(2 * b2 + b1);
        acc[grp * 16 + e] += cd(gd[r * R + r].re, gd[r * R + r].im);
      }
    }
    for (int i = 0; i < DI_GROUPS * 16; ++i) T.t[i] = cx{(real)acc[i].real(), (real)acc[i].imag()};
    return ng;
  }

  // --- backward (Circuit::backward, circuit.rs:266-429) --------------------------------------
  const char* backward(const Flat& dg, const Flat& cg, const Flat& vg, qdc_complex* out) {
    hclock::time_point ht[6];
    ht[0] = hclock::now();
    std::vector<size_t> gidx;
    QDC_TRY(validate_backward(dg, cg, vg, gidx));
    if (!dry) QDC_TRY(dyn_reset_all());
    const size_t nvar = n_var();
    for (auto& s : sh) {
      if (!s.bwd) {
        QDC_TRY(s.c().use());
        QDC_HIP(hipMalloc(&s.bwd, ((size_t)1 << nl) * sizeof(cx)));
        s.owned.push_back(s.bwd);
      }
      s.bwd_live = true;
    }
    // slots [0, nvar): per-gate gradients; [nvar, nvar + stages): fused stages' Gamma
    const size_t nslots = std::max<size_t>(2 * nvar, 1);
    if (!dry) QDC_TRY(ensure_out(false, nslots * RED));
    // variable gates met before the first cotangent keep zero gradients (circuit.rs:327-331)
    for (auto& s : sh) {
      QDC_TRY(s.c().use());
      QDC_HIP(hipMemsetAsync(s.grads, 0, sizeof(cx) * nslots * RED, s.c().stream));
    }
    std::vector<uint32_t> var_idx(ins.size(), 0);
    {
      uint32_t v = 0;
      for (size_t k = 0; k < ins.size(); ++k)
        if (is_var(ins[k].kind)) var_idx[k] = v++;
    }
    bool have_bwd = false;
    mark_inexact(cg, vg, gidx);
    ht[1] = hclock::now();
    std::vector<qdc_plan_op> pl;
    std::vector<Item> items;
    size_t first_inject = 0;
    // mirrored: the forward's passes in reverse, when this backward follows that forward with
    // the same gates (else the backward schedules itself)
    bool mirrored = false;
    if (mirror_on() && mrec.valid && mrec.inexact == inexact && mrec.end_phys == layout.phys) {
      const size_t nc = cg.size() ? cg.off.back() + cg.len.back() : 0;
      const size_t nv = vg.size() ? vg.off.back() + vg.len.back() : 0;
      const bool same = nc == mrec.cgates.size() && nv == mrec.vgates.size() &&
                        (nc == 0 || std::memcmp(cg.data, mrec.cgates.data(), nc * sizeof(qdc_complex)) == 0) &&
                        (nv == 0 || std::memcmp(vg.data, mrec.vgates.data(), nv * sizeof(qdc_complex)) == 0);
      mirrored = same && mirror_schedule(pl, items, first_inject);
    }
    mrec.valid = false;  // (this backward changes the layout and the state)
    if (!mirrored) {
      pl = plan(QDC_PLAN_BACKWARD);
      first_inject = pl.size();
      for (size_t i = 0; i < pl.size(); ++i)
        if (pl[i].type == QDC_PLAN_OP && is_diff_density(ins[pl[i].instr].kind)) {
          first_inject = i;
          break;
        }
      // QDC_MIRROR=2 (tests): a backward that cannot mirror its forward is an error
      if (mirror_on() && mirror == 2)
        return fail("mirror: the backward does not follow a forward call with the same gates");
      items = schedule(pl, true, first_inject);
    }
    if (diag_inject) merge_diag_injections(items, pl, dg, gidx);
    ht[2] = hclock::now();
    // a run of diagonal cotangent injections: one elementwise pass (no pass program)
    auto run_diag_inject = [&](const Item& item) -> const char* {
      diag_tab T;
      const uint32_t ng = diag_table(item, pl, dg, gidx, T);
      for (auto& s : sh) {
        QDC_TRY(s.c().use());
        QDC_TRY(qdc::diag_inject(s.c(), s.state, s.bwd, T, ng, nl, gm, have_bwd));
      }
      have_bwd = true;
      return nullptr;
    };
    // the backward's leading diagonal-injection passes need no program: they are launched
    // before it is built, so the device runs them during the host's build (round 6;
    // QDC_EARLY_INJECT=0: after)
    size_t lead = 0;
    if (!dry && early_inject)
      for (; lead < items.size() && items[lead].type == 3; ++lead) QDC_TRY(run_diag_inject(items[lead]));
    size_t mats_off = 0;
    const auto tb0 = std::chrono::steady_clock::now();
    QDC_TRY(build_program(items, pl, true, first_inject, cg, vg, gidx, mats_off, var_idx,
                          (uint32_t)nvar, {}, &dg));
    ht[3] = hclock::now();
    if (dry) return tracing ? trace_logical(items, pl, true, cg, vg, gidx) : nullptr;
    if (rq_stats)
      fprintf(stderr, "backward plan+build %.3f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count());
    for (size_t ii = lead; ii < items.size(); ++ii) {
      const Item& item = items[ii];
      if (item.type == 3) {
        QDC_TRY(run_diag_inject(item));
        continue;
      }
      if (item.type == 2) {
        const bool two = item.ops[0] >= first_inject;
        if (two && !have_bwd) {  // the first injection is fused: it adds into a zero bwd
          for (auto& s : sh) {
            QDC_TRY(s.c().use());
            QDC_TRY(zero_bwd(s));
          }
          have_bwd = true;
        }
        QDC_TRY(run_fused(item, two, mats_off, true));
        continue;
      }
      const qdc_plan_op& op = pl[item.ops[0]];
      if (op.type == QDC_PLAN_REMAP) {
        QDC_TRY(item.inv ? unremap(op, have_bwd) : remap(op, have_bwd));
        continue;
      }
      const Instr& in = ins[op.instr];
      if (is_const(in.kind) || is_var(in.kind)) {
        const bool var = is_var(in.kind);
        const qdc_complex* g4 = var ? vg.at(gidx[op.instr]) : cg.at(gidx[op.instr]);
        for (auto& s : sh) {
          Ctx& ctx = s.c();
          QDC_TRY(ctx.use());
          if (!have_bwd) {
            QDC_TRY(apply_gate(ctx, in, g4, s.state, op.pos2, op.pos1, true));
            continue;
          }
          cx* gbase = var ? s.grads : nullptr;
          const uint32_t dst = var_idx[op.instr];
          if (is_diag(in.kind)) {
            QDC_TRY(reverse_diag(ctx, s.state, s.bwd, to_diag(g4), op.pos2, op.pos1, nl, gbase, dst));
          } else if (is_q1_gate(in.kind)) {
            const mat<2> u = to_mat<2>(g4);
            mat<2> A;
            if (is_nonu(in.kind))
              QDC_TRY(inverse<2>(u, A));
            else
              A = conj_transpose<2>(u);
            QDC_TRY(reverse_dense<2>(ctx, s.state, s.bwd, A, transpose<2>(u), op.pos2, op.pos2, nl,
                                     gbase, dst));
          } else {
            const mat<4> u = to_mat<4>(g4);
            mat<4> A;
            if (is_nonu(in.kind))
              QDC_TRY(inverse<4>(u, A));
            else
              A = conj_transpose<4>(u);
            QDC_TRY(reverse_dense<4>(ctx, s.state, s.bwd, A, transpose<4>(u), op.pos2, op.pos1, nl,
                                     gbase, dst));
          }
        }
      } else {  // Diff density: inject its cotangent
        const qdc_complex* gd = dg.at(gidx[op.instr]);
        for (auto& s : sh) {
          Ctx& ctx = s.c();
          QDC_TRY(ctx.use());
          if (is_q1_density(in.kind))
            QDC_TRY(inject<2>(ctx, s.state, s.bwd, transpose<2>(to_mat<2>(gd)), op.pos2, op.pos2, nl,
                              !have_bwd));
          else
            QDC_TRY(inject<4>(ctx, s.state, s.bwd, transpose<4>(to_mat<4>(gd)), op.pos2, op.pos1, nl,
                              !have_bwd));
        }
        have_bwd = true;
      }
    }
    ht[4] = hclock::now();
    QDC_TRY(flush_all());
    const size_t used = nvar + stage_post.size();
    std::vector<cx*> bufs;
    for (auto& s : sh) bufs.push_back(s.grads);
    QDC_TRY(ex.allreduce(sh, bufs, used * RED));
    std::vector<int> widths;
    for (auto& in : ins)
      if (is_var(in.kind)) widths.push_back(gate_len(in.kind));
    QDC_TRY(collect(sh[0].grads, widths, out, used));
    // gradients of fused stages: G = ptrace(L Gamma Rt) per gate (qdc_stage.hpp)
    if (!stage_post.empty()) {
      std::vector<size_t> off(widths.size() + 1, 0);
      for (size_t j = 0; j < widths.size(); ++j) off[j + 1] = off[j] + widths[j];
      for (const StagePost& st : stage_post) {
        SMatD G = smat_identity<double>(st.R);
        const cx* g = host_out + (size_t)st.slot * RED;
        auto sw = [&](int p) { return st.swapped ? swap_bits4(p) : p; };
        if (st.diag_only) {
          for (int i = 0; i < 16; ++i) G.a[i] = 0;
          for (int r = 0; r < 4; ++r) G.a[r * 4 + r] = cdd(g[sw(r)].x, g[sw(r)].y);
        } else if (st.R == 4) {
          for (int p = 0; p < 4; ++p)
            for (int q = 0; q < 4; ++q) {
              const cx v = g[sw(p) * 4 + sw(q)];
              G.a[p * 4 + q] = cdd(v.x, v.y);
            }
        } else {
          for (int i = 0; i < st.R * st.R; ++i) G.a[i] = cdd(g[i].x, g[i].y);
        }
        for (const StageGate& sg : st.gates) {
          const SMatD M = smat_mul(smat_mul(sg.L, G), sg.Rt);
          cdd v[16];
          stage_extract(M, sg.diag, sg.role, v);
          qdc_complex* o = out + off[sg.var];
          for (int k = 0; k < widths[sg.var]; ++k) {
            o[k].re = (qdc_real)v[k].real();
            o[k].im = (qdc_real)v[k].imag();
          }
        }
      }
    }
    ht[5] = hclock::now();
    host_record(1, ht);
    return nullptr;
  }
};

}  // namespace qdc
