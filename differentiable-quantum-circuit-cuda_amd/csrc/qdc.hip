// qdc.hip — the single translation unit of libqdc_{f32,f64}.so.
//
// Build (see Makefile): hipcc -O3 --offload-arch=gfx950 -fPIC -shared [-DQDC_F64]
// Exports: the 18 reference primitives (include/qdc/primitives.h) and the circuit runtime
// (include/qdc/circuit.h).  Everything else has hidden visibility.
#include "qdc_circuit.hpp"
#include "qdc_primitives.hpp"
#include "qdc_spec.hpp"

// Build-time check of the specialized pass templates (qdc_spec.hpp): the runtime compiles their
// instances on the GPU box from these same headers; these (one exchange of each form) never run.
namespace {
template <int R>
struct SpecCheckTwo {
  __device__ __forceinline__ void operator()(qdc::cx (&xf)[R], qdc::cx (&xb)[R], const qdc::SpecEnv& E) const {
    constexpr uint32_t z[32] = {};
    qdc::spec_xchg_imm<6, false>(xf, E, z, z);
    qdc::spec_xchg<6, false>(xb, E, z, z, z, z);
  }
};
template <int R, int TB>
struct SpecCheckOne {
  __device__ __forceinline__ void operator()(qdc::cx (&x)[R], const qdc::SpecEnv& E) const {
    constexpr uint32_t z[32] = {};
    qdc::spec_xchg_imm<TB, true>(x, E, z, z);
    qdc::spec_xchg<TB, true>(x, E, z, z, z, z);
  }
};
}  // namespace
#define QDC_SPEC_CHECK(name, threads, pass)                                                       \
  __global__ __launch_bounds__(threads) void name(qdc::chunk* f, qdc::chunk* b, const qdc::fop* ops, \
                                                  const qdc::cx* mats, qdc::fgeo fg, uint32_t l0,    \
                                                  qdc::cx* partials, uint64_t slot_stride) {         \
    pass(f, b, ops, mats, fg, l0, partials, slot_stride);                                        \
  }
#ifndef QDC_F64
QDC_SPEC_CHECK(k_spec_check_two, 64, (qdc::rw_pass<true, 2, false, 1, true, SpecCheckTwo<32>>))
QDC_SPEC_CHECK(k_spec_check_one, 256, (qdc::rq_pass<false, 256, true, SpecCheckOne<16, 8>>))
#else
QDC_SPEC_CHECK(k_spec_check_two, 64, (qdc::rw_pass<true, 1, false, 1, false, SpecCheckTwo<16>>))
QDC_SPEC_CHECK(k_spec_check_one, 128, (qdc::rw_pass<false, 1, false, 2, false, SpecCheckOne<16, 7>>))
#endif
#undef QDC_SPEC_CHECK

struct qdc_circuit {
  qdc::Circuit impl;
};

#define QDC_API extern "C" __attribute__((visibility("default")))

static const char* new_circuit(qdc_circuit** out, size_t n, int world, int rank0, int nlocal,
                               ncclComm_t comm, const std::vector<int>* devices = nullptr,
                               const std::vector<ncclComm_t>* comms = nullptr);

QDC_API const char* qdc_circuit_new(qdc_circuit** out, size_t qubits_number) {
  return new_circuit(out, qubits_number, 1, 0, 1, nullptr);
}

QDC_API void qdc_circuit_free(qdc_circuit* c) {
  qdc::DeviceGuard keep;
  if (!c) return;
  c->impl.destroy();
  delete c;
}

QDC_API size_t qdc_circuit_qubits(const qdc_circuit* c) { return c->impl.n; }

QDC_API const char* qdc_circuit_set_state_from_vector(qdc_circuit* c, const qdc_complex* vec,
                                                      size_t len) {
  qdc::DeviceGuard keep;  // every entry point leaves the caller's device current
  // QuantizedTensor::set_from_host + get_qubits_number (quantized_tensor.rs:44-52, 76-80);
  // a sharded circuit takes its slices of the full vector (the initial layout is identity)
  qdc::Circuit& k = c->impl;
  if (len == 0 || (len & (len - 1)) != 0) return qdc::fail("State size is not a power of 2.");
  if (len != ((size_t)1 << k.n))
    return qdc::fail("Size of the given state does not match the size of the tensor.");
  const size_t shard = (size_t)1 << k.nl;
  k.initial_standard = false;
  for (size_t s = 0; s < k.sh.size(); ++s) {
    QDC_TRY(k.sh[s].c().use());
    QDC_HIP(hipMemcpyAsync(k.sh[s].initial, vec + (size_t)(k.ex.rank0 + s) * shard,
                           shard * sizeof(qdc_complex), hipMemcpyHostToDevice, k.sh[s].c().stream));
  }
  return k.sync_all();
}

QDC_API const char* qdc_circuit_push(qdc_circuit* c, int kind, size_t pos2, size_t pos1) {
  if (kind < QDC_CONST_Q2 || kind > QDC_DIFF_Q1_DENSITY)
    return qdc::fail("unknown instruction kind %d", kind);
  const bool q1 = qdc::is_q1_gate(kind) || qdc::is_q1_density(kind);
  c->impl.ins.push_back({kind, (uint32_t)pos2, q1 ? 0u : (uint32_t)pos1});
  // a backward after this push runs the new instruction too: the last forward's mirrored
  // schedule does not cover it (the backward then schedules itself)
  c->impl.mrec.valid = false;
  return nullptr;
}

QDC_API size_t qdc_circuit_len(const qdc_circuit* c) { return c->impl.ins.size(); }

QDC_API size_t qdc_circuit_output_size(const qdc_circuit* c, int mode) {
  return c->impl.output_size(mode);
}

QDC_API size_t qdc_circuit_grad_size(const qdc_circuit* c) { return c->impl.grad_size(); }

QDC_API const char* qdc_circuit_execute(qdc_circuit* c, int mode, const qdc_complex* cg,
                                        const size_t* cl, size_t nc, const qdc_complex* vg,
                                        const size_t* vl, size_t nv, qdc_complex* dens) {
  qdc::DeviceGuard keep;
  qdc::Flat cf(cg, cl, nc), vf(vg, vl, nv);
  return c->impl.execute(mode, cf, vf, dens);
}

QDC_API const char* qdc_circuit_backward(qdc_circuit* c, const qdc_complex* dg, const size_t* dl,
                                         size_t nd, const qdc_complex* cg, const size_t* cl,
                                         size_t nc, const qdc_complex* vg, const size_t* vl,
                                         size_t nv, qdc_complex* grads) {
  qdc::DeviceGuard keep;
  qdc::Flat df(dg, dl, nd), cf(cg, cl, nc), vf(vg, vl, nv);
  return c->impl.backward(df, cf, vf, grads);
}

QDC_API const char* qdc_circuit_get_shard(qdc_circuit* c, int which, int shard,
                                          qdc_complex* host, size_t len) {
  qdc::DeviceGuard keep;
  qdc::Circuit& k = c->impl;
  if (shard < 0 || (size_t)shard >= k.sh.size()) return qdc::fail("no local shard %d", shard);
  if (len != ((size_t)1 << k.nl)) return qdc::fail("shard length mismatch");
  const qdc::Shard& s = k.sh[shard];
  const qdc::cx* src = which == 0 ? s.state : which == 1 ? s.initial : s.bwd_live ? s.bwd : nullptr;
  if (!src) return qdc::fail("state %d is not allocated", which);
  QDC_TRY(k.sync_all());  // every shard's work, not only this shard's stream
  QDC_TRY(s.c().use());
  QDC_TRY(k.read_state(s, src, 0, host, len));
  QDC_HIP(hipStreamSynchronize(s.c().stream));
  return nullptr;
}

// A range of one local shard in physical order (no qubit un-permutation): for streaming reads
// of states too large for one host copy, e.g. the uncompute error of a 64 GiB state.
QDC_API const char* qdc_circuit_get_range(qdc_circuit* c, int which, int shard, size_t offset,
                                          qdc_complex* host, size_t len) {
  qdc::DeviceGuard keep;
  qdc::Circuit& k = c->impl;
  if (shard < 0 || (size_t)shard >= k.sh.size()) return qdc::fail("no local shard %d", shard);
  const size_t size = (size_t)1 << k.nl;
  if (offset > size || len > size - offset) return qdc::fail("range out of the shard");
  const qdc::Shard& s = k.sh[shard];
  const qdc::cx* src = which == 0 ? s.state : which == 1 ? s.initial : s.bwd_live ? s.bwd : nullptr;
  if (!src) return qdc::fail("state %d is not allocated", which);
  QDC_TRY(k.sync_all());
  QDC_TRY(s.c().use());
  QDC_TRY(k.read_state(s, src, offset, host, len));
  QDC_HIP(hipStreamSynchronize(s.c().stream));
  return nullptr;
}

// Unsharded circuits only (a sharded state is assembled from qdc_circuit_get_shard + layout).
QDC_API const char* qdc_circuit_get_state(qdc_circuit* c, int which, qdc_complex* host,
                                          size_t len) {
  qdc::Circuit& k = c->impl;
  if (k.g != 0) return qdc::fail("sharded state: use qdc_circuit_get_shard and qdc_circuit_layout");
  if (len != ((size_t)1 << k.n)) return qdc::fail("state length mismatch");
  QDC_TRY(qdc_circuit_get_shard(c, which, 0, host, len));
  // fused passes may leave fwd / bwd in a permuted qubit layout; `initial` never is
  bool ident = true;
  for (uint32_t q = 0; q < k.n; ++q) ident = ident && k.layout.phys[q] == q;
  if (which == 1 || ident) return nullptr;
  std::vector<qdc_complex> phys(host, host + len);
  // logical index i -> physical index: OR of per-11-bit-field tables
  constexpr uint32_t FB = 11;
  const uint32_t nf = (k.n + FB - 1) / FB;
  std::vector<std::vector<size_t>> tab(nf);
  for (uint32_t f = 0; f < nf; ++f) {
    const uint32_t lo = f * FB, w = std::min(FB, k.n - lo);
    tab[f].resize((size_t)1 << w);
    for (size_t v = 0; v < tab[f].size(); ++v) {
      size_t p = 0;
      for (uint32_t b = 0; b < w; ++b) p |= ((v >> b) & 1u) << k.layout.phys[lo + b];
      tab[f][v] = p;
    }
  }
  for (size_t i = 0; i < len; ++i) {
    size_t p = 0;
    for (uint32_t f = 0; f < nf; ++f) p |= tab[f][(i >> (f * FB)) & (tab[f].size() - 1)];
    host[i] = phys[p];
  }
  return nullptr;
}

// The whole physical state (every shard, global shard index = the top g physical bits) on
// every process: the local shards are copied, the others come from their processes by one RCCL
// broadcast each, staged through the remap scratch buffer (a shard of device memory, so no
// process needs the whole state on its GPU).  Collective over the circuit's communicator.
QDC_API const char* qdc_circuit_gather_state(qdc_circuit* c, int which, qdc_complex* host,
                                             size_t len) {
  qdc::DeviceGuard keep;
  qdc::Circuit& k = c->impl;
  if (len != ((size_t)1 << k.n)) return qdc::fail("state length mismatch");
  const size_t shard = (size_t)1 << k.nl;
  if (!k.ex.comm) {  // every shard is local
    if ((int)k.sh.size() != k.ex.world) return qdc::fail("shards of other processes need a communicator");
    for (size_t s = 0; s < k.sh.size(); ++s)
      QDC_TRY(qdc_circuit_get_shard(c, which, (int)s, host + s * shard, shard));
    return nullptr;
  }
  const qdc::Shard& s = k.sh[0];
  const qdc::cx* src = which == 0 ? s.state : which == 1 ? s.initial : s.bwd_live ? s.bwd : nullptr;
  // every rank takes the same path (which is the same everywhere), so none waits alone
  if (!src) return qdc::fail("state %d is not allocated", which);
  if (!s.scratch) return qdc::fail("no staging buffer");
  QDC_TRY(k.sync_all());
  QDC_TRY(s.c().use());
  const hipStream_t st = s.c().stream;
  for (int r = 0; r < k.ex.world; ++r) {
    QDC_NCCL(ncclBroadcast(src, s.scratch, shard * 2, qdc::Exchange::type(), r, k.ex.comm, st));
    QDC_HIP(hipMemcpyAsync(host + (size_t)r * shard, s.scratch, shard * sizeof(qdc_complex),
                           hipMemcpyDeviceToHost, st));
    QDC_HIP(hipStreamSynchronize(st));
  }
  return nullptr;
}

QDC_API const char* qdc_circuit_layout(const qdc_circuit* c, unsigned* phys, int* world,
                                       int* rank, int* local_shards) {
  const qdc::Circuit& k = c->impl;
  if (phys)
    for (uint32_t q = 0; q < k.n; ++q) phys[q] = k.layout.phys[q];
  if (world) *world = k.ex.world;
  if (rank) *rank = k.ex.rank0;
  if (local_shards) *local_shards = (int)k.sh.size();
  return nullptr;
}

// ---- communicator + sharded constructors ---------------------------------------------------
struct qdc_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  int device = 0;                 // the rank's GPU (current when the communicator was made)
  hipStream_t stream = nullptr;   // host-value collectives (qdc_comm_allreduce)
  double* dbuf = nullptr;         // their device staging, QDC_COMM_VALS doubles
};
constexpr int QDC_COMM_VALS = 64;

QDC_API const char* qdc_comm_unique_id(unsigned char id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  ncclUniqueId u;
  QDC_NCCL(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return nullptr;
}

QDC_API const char* qdc_comm_init(qdc_comm** out, int rank, int world,
                                  const unsigned char id[128]) {
  *out = nullptr;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  qdc_comm* c = new qdc_comm();
  c->rank = rank;
  c->world = world;
  if (hipGetDevice(&c->device) != hipSuccess) {
    delete c;
    return qdc::fail("qdc_comm_init: no current HIP device");
  }
  const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return qdc::fail("RCCL ERROR: ncclCommInitRank failed with %s.", ncclGetErrorString(r));
  }
  *out = c;
  return nullptr;
}

QDC_API void qdc_comm_free(qdc_comm* c) {
  if (!c) return;
  qdc::DeviceGuard keep;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// Sum (op 0) or maximum (op 1) of `count` host doubles over the communicator's ranks, in place
// on every rank; count 0 is a barrier.  Lets a one-process-per-GPU job time itself (bench.py's
// barrier and max over ranks) over the circuit's own RCCL communicator, without a second
// collective stack in the process.
QDC_API const char* qdc_comm_allreduce(qdc_comm* c, double* vals, int count, int op) {
  if (!c) return qdc::fail("no communicator");
  if (count < 0 || count > QDC_COMM_VALS) return qdc::fail("allreduce of %d values (max %d)", count, QDC_COMM_VALS);
  if (op != 0 && op != 1) return qdc::fail("allreduce op %d (0 sum, 1 max)", op);
  if (c->world == 1) return nullptr;
  qdc::DeviceGuard keep;
  QDC_HIP(hipSetDevice(c->device));
  if (!c->stream) QDC_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  if (!c->dbuf) QDC_HIP(hipMalloc(&c->dbuf, sizeof(double) * QDC_COMM_VALS));
  const int m = count > 0 ? count : 1;
  if (count > 0)
    QDC_HIP(hipMemcpyAsync(c->dbuf, vals, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
  else
    QDC_HIP(hipMemsetAsync(c->dbuf, 0, sizeof(double), c->stream));
  QDC_NCCL(ncclAllReduce(c->dbuf, c->dbuf, m, ncclDouble, op == 0 ? ncclSum : ncclMax, c->comm,
                         c->stream));
  if (count > 0)
    QDC_HIP(hipMemcpyAsync(vals, c->dbuf, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
  QDC_HIP(hipStreamSynchronize(c->stream));
  return nullptr;
}

static const char* new_circuit(qdc_circuit** out, size_t n, int world, int rank0, int nlocal,
                               ncclComm_t comm, const std::vector<int>* devices,
                               const std::vector<ncclComm_t>* comms) {
  *out = nullptr;
  QDC_TRY(qdc::check_n(n));
  qdc_circuit* c = new qdc_circuit();
  const char* e = c->impl.init((uint32_t)n, world, rank0, nlocal, comm, devices, comms);
  if (e) {
    c->impl.destroy();
    delete c;
    return e;
  }
  *out = c;
  return nullptr;
}

QDC_API const char* qdc_circuit_new_sharded(qdc_circuit** out, size_t n, qdc_comm* comm) {
  if (!comm) return qdc::fail("no communicator");
  return new_circuit(out, n, comm->world, comm->rank, 1, comm->world > 1 ? comm->comm : nullptr);
}

QDC_API const char* qdc_circuit_new_local_shards(qdc_circuit** out, size_t n, int shards) {
  if (shards < 1) return qdc::fail("shards must be >= 1");
  return new_circuit(out, n, shards, 0, shards, nullptr);
}

// One process, one shard per listed device (ncclCommInitAll over the node's
// GPUs, the single-process Python API of example_vqse_ising.py).  Distinct devices: RCCL
// communicators from ncclCommInitAll, collectives grouped over the shards' streams.  One device
// repeated: the shards share it, each on its own stream, exchanged by copies ordered with
// events (the same per-shard stream / context / program plumbing, on one GPU).
QDC_API const char* qdc_circuit_new_devices(qdc_circuit** out, size_t n, int ndev,
                                            const int* devices) {
  *out = nullptr;
  if (ndev < 1 || !devices) return qdc::fail("no devices");
  std::vector<int> devs(devices, devices + ndev);
  bool all_same = true, distinct = true;
  for (int i = 0; i < ndev; ++i)
    for (int j = 0; j < i; ++j) {
      all_same = all_same && devs[i] == devs[j];
      distinct = distinct && devs[i] != devs[j];
    }
  if (!all_same && !distinct)
    return qdc::fail("devices must be all distinct (RCCL) or all the same (one GPU)");
  int count = 0;
  QDC_HIP(hipGetDeviceCount(&count));
  for (int d : devs)
    if (d < 0 || d >= count) return qdc::fail("device %d does not exist (%d visible)", d, count);
  QDC_TRY(qdc::check_n(n));
  const uint32_t g = qdc::log2_exact((size_t)ndev);
  if (g == UINT32_MAX || g > 8 || (g > 0 && n < 2 * (size_t)g + 3))
    return qdc::fail("%d devices cannot shard %zu qubits (a power of two <= 256, n >= 2g + 3)",
                     ndev, n);
  qdc::DeviceGuard keep;
  std::vector<ncclComm_t> comms;
  if (ndev > 1 && distinct) {
    comms.resize(ndev);
    QDC_NCCL(ncclCommInitAll(comms.data(), ndev, devs.data()));
  }
  // from here the circuit owns the communicators (its destroy() frees them, also on error)
  return new_circuit(out, n, ndev, 0, ndev, nullptr, &devs, &comms);
}

// ---- planner -----------------------------------------------------------------------------
QDC_API size_t qdc_plan(size_t n, size_t world, const int* kinds, const unsigned* pos2,
                        const unsigned* pos1, size_t count, int mode, const unsigned* start_phys,
                        qdc_plan_op* out, size_t cap, unsigned* end_phys) {
  const uint32_t g = qdc::log2_exact(world);
  if (g == UINT32_MAX || n < 2 * (size_t)g + 3 || n > 64) return 0;
  std::vector<qdc::PlanIn> all(count);
  for (size_t i = 0; i < count; ++i) all[i] = {kinds[i], pos2[i], pos1[i]};
  std::vector<qdc::PlanIn> ops;
  std::vector<int> index;
  if (mode < QDC_PLAN_RUN || mode > QDC_PLAN_FORWARD_MIRROR) return 0;
  const bool mirror = mode == QDC_PLAN_FORWARD_MIRROR;
  qdc::active_ops(all, mirror ? (int)QDC_PLAN_FORWARD : mode, ops, index);
  qdc::QubitMap m;
  m.identity((uint32_t)n, g);
  if (start_phys) {
    for (uint32_t q = 0; q < n; ++q) m.phys[q] = start_phys[q];
    for (uint32_t q = 0; q < n; ++q) m.logi[m.phys[q]] = q;
  }
  std::vector<qdc_plan_op> plan;
  qdc::plan_pass(ops, index, m, plan, mode == QDC_PLAN_BACKWARD, nullptr, mirror);
  for (size_t i = 0; i < plan.size() && i < cap; ++i) out[i] = plan[i];
  if (end_phys)
    for (uint32_t q = 0; q < n; ++q) end_phys[q] = m.phys[q];
  return plan.size();
}

QDC_API const char* qdc_circuit_sync(qdc_circuit* c) {
  qdc::DeviceGuard keep;
  return c->impl.sync_all();
}

QDC_API const char* qdc_circuit_profile(qdc_circuit* c, int on) {
  qdc::DeviceGuard keep;
  for (auto& d : c->impl.devs) {
    qdc::Ctx& x = d->ctx;
    if (on) {
      QDC_TRY(x.sync());
      x.prof.reset();
    }
    x.prof.on = on != 0;
  }
  return nullptr;
}

// launches of every device context (a kernel's count and time summed over the devices)
QDC_API size_t qdc_circuit_profile_collect(qdc_circuit* c, qdc_kernel_stat* out, size_t cap) {
  std::vector<qdc::Ctx*> xs;
  for (auto& d : c->impl.devs) xs.push_back(&d->ctx);
  return qdc::prof_collect(xs, out, cap);
}

// Host time of the circuit's calls since the last reset: out[0..5] run/forward, out[6..11]
// backward, each (calls, setup ms, schedule ms, program-build ms, launch ms, finish ms: stream
// sync, result copies and gradient reconstruction).  Returns the values written.
QDC_API size_t qdc_circuit_host_times(qdc_circuit* c, double* out, size_t n, int reset) {
  size_t k = 0;
  for (int d = 0; d < 2; ++d)
    for (int j = 0; j < 6; ++j, ++k)
      if (out && k < n) out[k] = c->impl.host_ms[d][j];
  if (reset)
    for (auto& row : c->impl.host_ms)
      for (double& v : row) v = 0;
  return std::min<size_t>(n, 12);
}

QDC_API const char* qdc_build_info(void) {
#ifdef QDC_F64
  return "qdc f64 gfx950";
#else
  return "qdc f32 gfx950";
#endif
}

QDC_API size_t qdc_fusion_schedule(size_t local_qubits, int backward, size_t first_inject,
                                   const int* kinds, const unsigned char* inexact,
                                   size_t n_instr, const qdc_plan_op* plan, size_t n_plan,
                                   int lcmin, int max_ops, unsigned* item_info, size_t item_cap,
                                   unsigned* stage_len, size_t stage_cap, unsigned* op_order,
                                   size_t op_cap) {
  std::vector<qdc::Instr> ins(n_instr);
  for (size_t k = 0; k < n_instr; ++k) ins[k] = qdc::Instr{kinds[k], 0, 0};
  std::vector<uint8_t> sens(n_instr, 0);
  if (inexact)
    for (size_t k = 0; k < n_instr; ++k) sens[k] = inexact[k] ? 1 : 0;
  qdc::FusionPlanner P{ins, sens, (uint32_t)local_qubits, true, true,
                             max_ops > 0 ? (uint32_t)std::min(max_ops, qdc::FMAX_OPS)
                                         : (uint32_t)qdc::FMAX_OPS,
                             lcmin > 0 ? (uint32_t)lcmin : 3u};
  if (const char* e = getenv("QDC_TILE2_CHUNKS")) P.tile2_chunks = (uint32_t)atoi(e);
  if (const char* e = getenv("QDC_TILE1_CHUNKS")) P.tile1_chunks = (uint32_t)atoi(e);
  // the runtime's f32 register-resident settings (qdc_circuit.hpp planner())
  if (const char* e = getenv("QDC_SCHED_RQ")) P.permute = P.rq_grad = atoi(e) != 0;
  if (const char* e = getenv("QDC_SCHED_PERM")) P.permute = atoi(e) != 0;  // f64: rq_grad only
  if (const char* e = getenv("QDC_SCHED_MIRROR")) P.mirror = atoi(e) != 0;  // QDC_MIRROR's forward
  if (const char* e = getenv("QDC_DEFER_Q1")) P.defer_q1 = atoi(e) != 0;
  if (const char* e = getenv("QDC_RQ_PERM_LOW")) P.perm_low = (uint32_t)atoi(e);
  if (const char* e = getenv("QDC_RQ_GSTAGE")) P.gamma_stage_cap = atoi(e) != 0;
  if (const char* e = getenv("QDC_DENS_SPLIT")) P.split_dens = atoi(e) != 0;
  std::vector<qdc_plan_op> pl(plan, plan + n_plan);
  const std::vector<qdc::FusionItem> items = P.fuse_items(pl, backward != 0, first_inject);
  size_t ns = 0, no = 0;
  for (size_t i = 0; i < items.size(); ++i) {
    const qdc::FusionItem& it = items[i];
    std::vector<std::vector<uint32_t>> stages;
    if (it.type == 2)
      stages = P.stage_partition(it.ops, pl, backward != 0);
    else
      stages.push_back(it.ops);
    if (i >= item_cap || ns + stages.size() > stage_cap) return SIZE_MAX;
    unsigned* info = item_info + 12 * i;
    info[0] = (unsigned)it.type;
    info[1] = (unsigned)stages.size();
    info[2] = it.lc;
    info[3] = it.h;
    for (int k = 0; k < 8; ++k) info[4 + k] = k < (int)qdc::FMAX_ROWS ? it.hb[k] : 0u;
    for (const auto& st : stages) {
      stage_len[ns++] = (unsigned)st.size();
      for (uint32_t op : st) {
        if (no >= op_cap) return SIZE_MAX;
        op_order[no++] = op;
      }
    }
  }
  return items.size();
}

QDC_API int qdc_gate_plan(unsigned n, unsigned R, unsigned pos2, unsigned pos1,
                          int two_states, int far_tile, unsigned* out) {
  if (!out || (R != 2 && R != 4) || n < 2 || n > 62 || pos2 >= n || pos1 >= n ||
      (R == 2 && pos2 != pos1) || (R == 4 && pos2 == pos1))
    return -1;
  const qdc::Plan p = qdc::plan_gate(n, (int)R, pos2, pos1, two_states != 0, 1024u, far_tile != 0);
  const uint64_t cnt = p.tile ? p.tg.ntiles : p.g.items;
  const unsigned v[10] = {p.tile ? 1u : 0u, (unsigned)p.mode, p.tg.l, p.tg.h, p.tg.hb0, p.tg.hb1,
                          p.tg.t1, p.tg.t2, (unsigned)(cnt & 0xffffffffu), (unsigned)(cnt >> 32)};
  for (int i = 0; i < 10; ++i) out[i] = v[i];
  return 0;
}

// Host-only test hook of the LANE family's geometry (plan_lane): out[0..9] = {ampk + 1, nlow,
// nf, f0, f1, m0, m1, units lo, units hi, it} for grid target 2048; reduces bit 1: the
// block-wide variant (1024-chunk units).  Returns -1 on bad arguments, 1 when the state is too
// small for the family.
QDC_API int qdc_lane_plan(unsigned n, unsigned R, unsigned pos2, unsigned pos1, int reduces,
                          unsigned* out) {
  if (!out || (R != 2 && R != 4) || n < 2 || n > 62 || pos2 >= n || pos1 >= n ||
      (R == 2 && pos2 != pos1) || (R == 4 && pos2 == pos1))
    return -1;
  qdc::Plan p;
  if (!qdc::plan_lane(n, (int)R, pos2, pos1, 2048u, (reduces & 1) != 0, p, 1, (reduces & 2) ? 10u : 6u))
    return 1;
  const qdc::lgeo& g = p.lg;
  const unsigned v[10] = {(unsigned)(p.ampk + 1), g.nlow, g.nf, g.f0, g.f1, g.m0, g.m1,
                          (unsigned)(g.units & 0xffffffffu), (unsigned)(g.units >> 32), g.it};
  for (int i = 0; i < 10; ++i) out[i] = v[i];
  return 0;
}

// Host-only test hook of the specialized passes (qdc_jit.hpp): plan a pass over n stages (as
// qdc_rq_plan; a two-state pass's stages all Gamma stages) on the runtime's tile of the
// precision, write its kernel source and compile it with hipcc for gfx950 (not loaded).  name_out receives the kernel name
// and, after a NUL, the code object's path.  Returns nullptr or an error message.
// the specialized kernel (name, source) of one pass program over n stages (qdc_spec_selftest)
static const char* spec_program_for(unsigned tile_bits, const unsigned* kinds, const unsigned* t1,
                                    const unsigned* t2, const unsigned long long* deps, size_t n,
                                    std::string& name, std::string& src) {
  if (n == 0 || n > 64) return "invalid arguments";
  std::vector<qdc::RqStage> st(n);
  for (size_t i = 0; i < n; ++i) st[i] = qdc::RqStage{kinds[i], t1[i], t2[i], deps ? deps[i] : 0};
  // the runtime's tiles: f32 11 two-state (five slots), 12 one-state; f64 10 two-state, 11 one-state;
  // tile_bits | 0x100: a one-state pass on the two-state tile size (f32: one wave, five slots)
  // | 0x200 as well: that pass prefetching the next tile (f32 one-wave: k_rw<false, 2, true, 1, true>)
  const bool force_one = (tile_bits & 0x100u) != 0, pf = (tile_bits & 0x200u) != 0;
  const unsigned tile_bits_in = tile_bits;
  tile_bits &= 0xffu;
  const unsigned t2bits = sizeof(qdc::real) == 4 ? 11u : 10u;
  if (tile_bits != t2bits && tile_bits != t2bits + 1) return "tile_bits: not a specialized pass's tile";
  const bool two = tile_bits == t2bits && !force_one;
  const qdc::SpecKind K = two ? qdc::spec_kind_two() : qdc::spec_kind_one(tile_bits, pf);
  const bool keep = K.ns == 5 && tile_bits == 11 && !pf && !(tile_bits_in & 0x400u) &&
                    sizeof(qdc::real) == 4;  // (as the runtime's spec_half planning)
  const qdc::RqPlan plan = qdc::rq_plan(st, tile_bits, nullptr, true, K.ns, keep);
  std::vector<qdc::SpecStep> sst;
  qdc::RqLayout cur = plan.load;
  for (const qdc::RqStep& s : plan.steps) {
    qdc::fop F{};
    if (s.relayout) {
      F.kind = qdc::FK_RELAYOUT;
      sst.push_back(qdc::SpecStep{true, cur, s.L, F});
      cur = s.L;
      continue;
    }
    F.kind = st[s.stage].kind | (two ? qdc::FOP_GAMMA : 0u);
    F.t1 = s.cs;
    const uint32_t kd = st[s.stage].kind;
    if ((kd == qdc::FK_Q2 || kd == qdc::FK_DIAG) && (s.cs >> 3) > (s.cs & 7u))
      F.t1 = (s.cs & 7u) * 8u + (s.cs >> 3);  // the runtime's canonical S1 < S2
    sst.push_back(qdc::SpecStep{false, cur, cur, F});
  }
  // (the runtime's choice: a one-wave one-state program whose relayouts all keep a slot runs on
  // half buffers, qdc_circuit.hpp half1; | 0x400 keeps the full buffer)
  const bool half = keep && qdc::spec_half_ok(sst);
  const qdc::SpecKind KK = !half ? K : two ? qdc::spec_kind_two(true) : qdc::spec_kind_one(tile_bits, false, true);
  const std::string body = qdc::spec_program_source(sst, tile_bits, KK);
  name = qdc::spec_kernel_name(body, KK);
  src = qdc::spec_kernel_source(name, body, KK);
  return nullptr;
}

QDC_API const char* qdc_spec_selftest(unsigned tile_bits, const unsigned* kinds, const unsigned* t1,
                                      const unsigned* t2, const unsigned long long* deps, size_t n,
                                      char* name_out, size_t cap) {
  if (!name_out || cap < 128) return "invalid arguments";
  std::string name, src;
  if (const char* e = spec_program_for(tile_bits, kinds, t1, t2, deps, n, name, src)) return e;
  if (const char* e = qdc::SpecJit::get().compile_only({name}, {src})) return e;
  const std::string obj = qdc::SpecJit::get().code_object(name);
  if (name.size() + obj.size() + 2 > cap) return "name buffer too small";
  std::memcpy(name_out, name.c_str(), name.size() + 1);
  std::memcpy(name_out + name.size() + 1, obj.c_str(), obj.size() + 1);
  return nullptr;
}

QDC_API const char* qdc_spec_selftest_batch(unsigned tile_bits, const size_t* counts, size_t nprog,
                                            const unsigned* kinds, const unsigned* t1,
                                            const unsigned* t2, const unsigned long long* deps,
                                            char* names_out, size_t cap) {
  if (!counts || !names_out || nprog == 0) return "invalid arguments";
  std::vector<std::string> names(nprog), srcs(nprog);
  size_t off = 0;
  for (size_t p = 0; p < nprog; ++p) {
    if (const char* e = spec_program_for(tile_bits, kinds + off, t1 + off, t2 + off,
                                         deps ? deps + off : nullptr, counts[p], names[p], srcs[p]))
      return e;
    off += counts[p];
  }
  if (const char* e = qdc::SpecJit::get().compile_only(names, srcs)) return e;
  size_t w = 0;
  for (const std::string& nm : names) {
    if (w + nm.size() + 1 > cap) return "name buffer too small";
    std::memcpy(names_out + w, nm.c_str(), nm.size() + 1);
    w += nm.size() + 1;
  }
  return nullptr;
}

// Ahead-of-time compilation of a circuit's specialized passes (build time, no GPU): a host-only
// dry run of forward(cg, vg) then backward(dg, cg, vg) on `world` shards builds the same pass
// programs as the runtime's calls, and every specialized kernel they would launch is compiled
// into the cache directory (QDC_JIT_DIR).  *kernels: the distinct kernels of the two calls.
QDC_API const char* qdc_precompile(size_t n, int world, const int* kinds, const unsigned* pos2,
                                   const unsigned* pos1, size_t count, const qdc_complex* cg,
                                   const size_t* cl, size_t nc, const qdc_complex* vg,
                                   const size_t* vl, size_t nv, const qdc_complex* dg,
                                   const size_t* dl, size_t nd, size_t* kernels) {
  if (n == 0 || n > 40 || world < 1) return qdc::fail("invalid precompile arguments");
  qdc::Circuit k;
  QDC_TRY(k.init_dry((uint32_t)n, world));
  for (size_t i = 0; i < count; ++i) {
    const int kind = kinds[i];
    if (kind < QDC_CONST_Q2 || kind > QDC_DIFF_Q1_DENSITY)
      return qdc::fail("unknown instruction kind %d", kind);
    const bool q1 = qdc::is_q1_gate(kind) || qdc::is_q1_density(kind);
    k.ins.push_back({kind, pos2[i], q1 ? 0u : pos1[i]});
  }
  qdc::Flat cf(cg, cl, nc), vf(vg, vl, nv), df(dg, dl, nd);
  std::vector<qdc_complex> dens(std::max<size_t>(k.output_size(QDC_MODE_FORWARD), 1));
  QDC_TRY(k.execute(QDC_MODE_FORWARD, cf, vf, dens.data()));
  std::vector<qdc_complex> grads(std::max<size_t>(k.grad_size(), 1));
  QDC_TRY(k.backward(df, cf, vf, grads.data()));
  std::vector<std::string> names, srcs;
  for (const qdc::SpecEntry* e : k.dry_specs) {
    names.push_back(e->name);
    srcs.push_back(e->src);
  }
  if (kernels) *kernels = names.size();
  // (QDC_PRECOMPILE_DUMP=dir: also write each kernel's source to dir/<name>.hip, in launch order
  // of first use, with dir/order.txt — the per-pass time model joins them with a kernel trace)
  if (const char* dd = getenv("QDC_PRECOMPILE_DUMP")) {
    const std::string d(dd);
    FILE* lst = fopen((d + "/order.txt").c_str(), "a");
    for (size_t i = 0; i < names.size(); ++i) {
      if (FILE* f = fopen((d + "/" + names[i] + ".hip").c_str(), "w")) {
        fwrite(srcs[i].data(), 1, srcs[i].size(), f);
        fclose(f);
      }
      if (lst) fprintf(lst, "%s\n", names[i].c_str());
    }
    if (lst) fclose(lst);
  }
  // (QDC_PRECOMPILE_COUNT=1: count the kernels only)
  const char* co = getenv("QDC_PRECOMPILE_COUNT");
  if (names.empty() || (co && atoi(co) != 0)) return nullptr;
  return qdc::SpecJit::get().compile_only(names, srcs);
}

// host-only hooks (qdc_trace_program, qdc_check_schedule): an instruction's kind and positions
// as qdc_circuit_push accepts them (positions < n, a two-qubit op's two positions distinct)
static const char* check_instr(int kind, unsigned p2, unsigned p1, size_t n, size_t i) {
  if (kind < QDC_CONST_Q2 || kind > QDC_DIFF_Q1_DENSITY)
    return qdc::fail("unknown instruction kind %d", kind);
  const bool q1 = qdc::is_q1_gate(kind) || qdc::is_q1_density(kind);
  if (p2 >= n || (!q1 && (p1 >= n || p1 == p2)))
    return qdc::fail("instruction %zu: invalid positions (%u, %u) on %zu qubits", i, p2, p1, n);
  return nullptr;
}

QDC_API const char* qdc_trace_program(size_t n, int world, const int* kinds, const unsigned* pos2,
                                      const unsigned* pos1, size_t count, const qdc_complex* cg,
                                      const size_t* cl, size_t nc, const qdc_complex* vg,
                                      const size_t* vl, size_t nv, const qdc_complex* dg,
                                      const size_t* dl, size_t nd, qdc_trace_op* out, size_t cap,
                                      size_t* n_out) {
  static_assert(sizeof(qdc_trace_op) == sizeof(qdc::Circuit::TraceOp), "trace op layout");
  if (n == 0 || n > 40 || world < 1 || !n_out || (count > 0 && (!kinds || !pos2 || !pos1)))
    return qdc::fail("invalid trace arguments");
  qdc::Circuit k;
  QDC_TRY(k.init_dry((uint32_t)n, world));
  for (size_t i = 0; i < count; ++i) {
    const int kind = kinds[i];
    if (const char* e = check_instr(kind, pos2[i], pos1[i], n, i)) return e;
    const bool q1 = qdc::is_q1_gate(kind) || qdc::is_q1_density(kind);
    k.ins.push_back({kind, pos2[i], q1 ? 0u : pos1[i]});
  }
  k.tracing = true;
  qdc::Flat cf(cg, cl, nc), vf(vg, vl, nv), df(dg, dl, nd);
  std::vector<qdc_complex> dens(std::max<size_t>(k.output_size(QDC_MODE_FORWARD), 1));
  QDC_TRY(k.execute(QDC_MODE_FORWARD, cf, vf, dens.data()));
  std::vector<qdc_complex> grads(std::max<size_t>(k.grad_size(), 1));
  QDC_TRY(k.backward(df, cf, vf, grads.data()));
  *n_out = k.trace.size();
  for (size_t i = 0; i < k.trace.size() && i < cap; ++i)
    std::memcpy(&out[i], &k.trace[i], sizeof(qdc_trace_op));
  return nullptr;
}

// Host-only consistency check of the runtime's forward schedule (tests): plan the forward of a
// circuit over `world` shards (mirrored when QDC_MIRROR is on, as the runtime does), fuse it
// (permuting passes relabel later remaps on sharded circuits), then replay the layout: every
// op's positions must be where its logical qubits are, every remap's victims local and
// ascending.  *items / *swaps (nullable): the schedule's items and permuting swaps.
QDC_API const char* qdc_check_schedule(size_t n, int world, const int* kinds, const unsigned* pos2,
                                       const unsigned* pos1, size_t count, size_t* items_out,
                                       size_t* swaps_out) {
  if (n == 0 || n > 40 || world < 1 || (count > 0 && (!kinds || !pos2 || !pos1)))
    return qdc::fail("invalid schedule arguments");
  qdc::Circuit k;
  QDC_TRY(k.init_dry((uint32_t)n, world));
  for (size_t i = 0; i < count; ++i) {
    if (const char* e = check_instr(kinds[i], pos2[i], pos1[i], n, i)) return e;
    const bool q1 = qdc::is_q1_gate(kinds[i]) || qdc::is_q1_density(kinds[i]);
    k.ins.push_back({kinds[i], pos2[i], q1 ? 0u : pos1[i]});
  }
  k.inexact.assign(k.ins.size(), 0);
  std::vector<qdc_plan_op> pl = k.plan(QDC_MODE_FORWARD);
  k.sched_mirror = true;
  const std::vector<qdc::Circuit::Item> items = k.schedule(pl, false, SIZE_MAX);
  qdc::QubitMap m;
  m.identity((uint32_t)n, k.g);
  size_t nsw = 0;
  for (const auto& it : items) {
    for (uint32_t pi : it.ops) {
      const qdc_plan_op& op = pl[pi];
      if (op.type == QDC_PLAN_REMAP) {
        for (uint32_t j = 0; j < op.nvictims; ++j) {
          if (op.victims[j] == 0 || op.victims[j] >= k.nl || (j > 0 && op.victims[j] <= op.victims[j - 1]))
            return qdc::fail("remap %u: victims not local, nonzero and ascending", pi);
        }
        m.apply(op.victims);
        continue;
      }
      const qdc::Instr& in = k.ins[op.instr];
      const bool q1 = qdc::is_q1_gate(in.kind) || qdc::is_q1_density(in.kind);
      if (op.pos2 != m.phys[in.a] || (!q1 && op.pos1 != m.phys[in.b]) || op.pos2 >= k.nl ||
          op.pos1 >= k.nl)
        return qdc::fail("plan op %u (instruction %d) at (%u, %u), its qubits at (%u, %u)", pi,
                         op.instr, op.pos2, op.pos1, m.phys[in.a], q1 ? m.phys[in.a] : m.phys[in.b]);
    }
    for (const auto& sw : it.swaps) m.swap_phys(sw.first, sw.second);
    nsw += it.swaps.size();
  }
  if (items_out) *items_out = items.size();
  if (swaps_out) *swaps_out = nsw;
  return nullptr;
}

QDC_API size_t qdc_jit_stats(double* stats, size_t n) {
  const qdc::JitStats s = qdc::SpecJit::get().counters();
  const bool on = qdc::SpecJit::get().enabled();
  const double v[9] = {(double)s.compiled, (double)s.waited, (double)s.loaded, s.compile_s,
                       s.wait_s, s.ensure_s, on ? 1.0 : 0.0,
                       (double)qdc::Ctx::spec_launches().load(std::memory_order_relaxed),
                       (double)s.queued};
  size_t k = 0;
  for (; stats && k < n && k < 9; ++k) stats[k] = v[k];
  return k;
}

QDC_API size_t qdc_jit_wait(double timeout_s) { return qdc::SpecJit::get().wait_async(timeout_s); }

QDC_API const char* qdc_jit_dir(char* dir_out, size_t cap) {
  if (!dir_out || cap < 2) return "invalid arguments";
  const std::string d = qdc::SpecJit::get().cache_dir();
  if (d.empty()) return "specialized passes are off (see the message on stderr)";
  if (d.size() + 1 > cap) return "buffer too small";
  std::memcpy(dir_out, d.c_str(), d.size() + 1);
  return nullptr;
}

QDC_API const char* qdc_spec_fingerprint(const char* defines, const char* compiler,
                                         const char* csrc_dir, unsigned long long* fingerprint,
                                         unsigned long long* source_hash) {
  if (!compiler || !csrc_dir || !fingerprint) return "invalid arguments";
  uint64_t sfp = 0;
  const std::string cs = csrc_dir;
  if (!qdc::spec_source_fp(cs, cs + "/../../include", sfp)) return "cannot read the kernel headers";
  *fingerprint = qdc::spec_fingerprint(defines ? std::string(defines) : qdc::spec_defines(), compiler, sfp);
  if (source_hash) *source_hash = sfp;
  return nullptr;
}

QDC_API size_t qdc_rq_plan(unsigned tile_bits, unsigned slots, const unsigned* kinds,
                           const unsigned* t1, const unsigned* t2,
                           const unsigned long long* deps, size_t n, unsigned* steps,
                           size_t cap) {
  if (n > 64) return SIZE_MAX;  // rq_plan's stage sets are 64-bit masks (passes hold <= FMAX_OPS)
  if (slots != 4 && slots != 5) return SIZE_MAX;
  std::vector<qdc::RqStage> st(n);
  for (size_t i = 0; i < n; ++i) st[i] = qdc::RqStage{kinds[i], t1[i], t2[i], deps ? deps[i] : 0};
  const char* mc = getenv("QDC_RQ_MAXCL");  // the runtime's knob (qdc_circuit.hpp)
  const char* kp = getenv("QDC_RQ_KEEP");  // (tests: the half-buffer planning, rq_plan keep)
  const qdc::RqPlan plan = qdc::rq_plan(st, tile_bits, nullptr, !(mc && atoi(mc) == 0), slots,
                                        kp && atoi(kp) != 0);
  if (plan.steps.size() + 2 > cap) return SIZE_MAX;
  auto put = [&](size_t i, unsigned kind, unsigned stage, unsigned cs, const qdc::RqLayout& L) {
    unsigned* o = steps + 8 * i;
    o[0] = kind;
    o[1] = stage;
    o[2] = cs;
    for (int s = 0; s < qdc::RQ_SLOTS_MAX; ++s) o[3 + s] = (unsigned)s < L.ns ? L.slot[s] : ~0u;
  };
  put(0, 2u, 0u, 0u, plan.load);
  for (size_t i = 0; i < plan.steps.size(); ++i)
    put(i + 1, plan.steps[i].relayout ? 1u : 0u, plan.steps[i].stage, plan.steps[i].cs,
        plan.steps[i].L);
  put(plan.steps.size() + 1, 3u, 0u, 0u, plan.store);
  return plan.steps.size() + 2;
}
