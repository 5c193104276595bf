// qdc_primitives.hpp — the 18 reference C-ABI entry points (src/primitives_bind.rs:15-119,
// implemented for CUDA in src/primitives.cu:141-953) on the HIP kernels.
//
// Every call runs on a context of the device that is current for the calling thread (as the
// reference launches on the current device's legacy default stream): one non-blocking stream
// per device, ordered exactly like that default stream; host results (copies, densities,
// gradients) synchronise it.  A host that switches devices (hipSetDevice) between calls, or
// drives one GPU per thread, gets each device's own stream and scratch.  A mutex makes
// concurrent callers safe (the reference's are not, README.md:13).
#pragma once

#include "qdc/circuit.h"
#include "qdc/dense.h"
#include "qdc_device.hpp"
#include "qdc_qk.hpp"

namespace qdc {

inline std::mutex& abi_mutex() {
  static std::mutex m;
  return m;
}

constexpr int ABI_MAX_DEVICES = 64;

inline const char* abi_ctx(Ctx*& out) {
  static Ctx* ctx[ABI_MAX_DEVICES] = {};
  int dev = 0;
  QDC_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= ABI_MAX_DEVICES) return fail("device %d is out of the supported range", dev);
  if (!ctx[dev]) {
    Ctx* c = new Ctx();
    const char* e = c->init(dev);
    if (e) {
      delete c;
      return e;
    }
    ctx[dev] = c;
  }
  out = ctx[dev];
  return nullptr;
}

inline const char* check_n(size_t n) {
  if (n > 40) return fail("qubits_number %zu is out of the supported range (<= 40).", n);
  return nullptr;
}

// one reduction → host `out[0..K)` += result (the reference's `+=`, primitives.cu:281-288)
inline const char* abi_finish_reduction(Ctx& c, qdc_complex* out, int K) {
  QDC_TRY(c.flush());
  QDC_HIP(hipMemcpyAsync(c.host_results, c.results, sizeof(cx) * RED, hipMemcpyDeviceToHost,
                         c.stream));
  QDC_HIP(hipStreamSynchronize(c.stream));
  for (int k = 0; k < K; ++k) {
    out[k].re += c.host_results[k].x;
    out[k].im += c.host_results[k].y;
  }
  return nullptr;
}

// per-kernel sums of a context's profiled launches (qdc_circuit_profile_collect,
// qdc_abi_profile_collect)
inline size_t prof_collect(const std::vector<Ctx*>& xs, qdc_kernel_stat* out, size_t cap) {
  std::vector<qdc_kernel_stat> agg;
  for (Ctx* x : xs) {
    (void)x->sync();
    for (auto& r : x->prof.recs) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) ms = 0.f;
      qdc_kernel_stat* s = nullptr;
      for (auto& a : agg)
        if (strncmp(a.name, r.name, sizeof(a.name)) == 0) s = &a;
      if (!s) {
        agg.push_back({});
        s = &agg.back();
        strncpy(s->name, r.name, sizeof(s->name) - 1);
      }
      s->launches += 1;
      s->total_ms += ms;
      s->algo_bytes += r.bytes;
      s->algo_flops += r.flops;
    }
  }
  for (size_t i = 0; i < agg.size() && i < cap; ++i) out[i] = agg[i];
  return agg.size();
}
inline size_t prof_collect(Ctx& x, qdc_kernel_stat* out, size_t cap) {
  return prof_collect(std::vector<Ctx*>{&x}, out, cap);
}

}  // namespace qdc

#define QDC_ABI_BEGIN                                   \
  std::lock_guard<std::mutex> qdc_lock_(qdc::abi_mutex()); \
  qdc::Ctx* ctxp = nullptr;                             \
  QDC_TRY(qdc::abi_ctx(ctxp));                          \
  qdc::Ctx& ctx = *ctxp;

#define QDC_VOID(expr)                                                  \
  do {                                                                  \
    const char* qdc_v_ = (expr);                                        \
    if (qdc_v_) fprintf(stderr, "qdc: %s\n", qdc_v_);                   \
  } while (0)

static const char* set2standard_impl(qdc_complex* state, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  return qdc::set_standard(ctx, reinterpret_cast<qdc::cx*>(state), (uint32_t)n);
}

static const char* check_q2(size_t pos2, size_t pos1, size_t n) {
  if (pos1 == pos2) return qdc::fail("pos1 and pos2 must be different.");
  if (pos1 >= n) return qdc::fail("pos1 is out of the bound.");
  if (pos2 >= n) return qdc::fail("pos2 is out of the bound.");
  return nullptr;
}

template <int OP>
static const char* elementwise_impl(const qdc_complex* src, qdc_complex* dst, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  return qdc::elementwise<OP>(ctx, reinterpret_cast<const qdc::cx*>(src),
                              reinterpret_cast<qdc::cx*>(dst), (uint32_t)n);
}

extern "C" {

__attribute__((visibility("default"))) void set2standard(qdc_complex* state, size_t n) {
  QDC_VOID(set2standard_impl(state, n));
}

__attribute__((visibility("default"))) const char* get_state(qdc_complex** state, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  (void)ctx;
  QDC_HIP(hipMalloc(reinterpret_cast<void**>(state), ((size_t)1 << n) * sizeof(qdc_complex)));
  return nullptr;
}

__attribute__((visibility("default"))) const char* drop_state(qdc_complex* state) {
  QDC_ABI_BEGIN
  QDC_HIP(hipStreamSynchronize(ctx.stream));
  QDC_HIP(hipFree(state));
  return nullptr;
}

__attribute__((visibility("default"))) const char* copy_to_host(const qdc_complex* state,
                                                                qdc_complex* host, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_HIP(hipMemcpyAsync(host, state, ((size_t)1 << n) * sizeof(qdc_complex),
                         hipMemcpyDeviceToHost, ctx.stream));
  QDC_HIP(hipStreamSynchronize(ctx.stream));
  return nullptr;
}

__attribute__((visibility("default"))) const char* set_from_host(qdc_complex* dev,
                                                                 const qdc_complex* host,
                                                                 size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_HIP(hipMemcpyAsync(dev, host, ((size_t)1 << n) * sizeof(qdc_complex),
                         hipMemcpyHostToDevice, ctx.stream));
  QDC_HIP(hipStreamSynchronize(ctx.stream));
  return nullptr;
}

__attribute__((visibility("default"))) const char* q1gate(qdc_complex* state,
                                                          const qdc_complex* gate, size_t pos,
                                                          size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  if (pos >= n) return qdc::fail("pos is out of the bound.");
  return qdc::apply_dense<2>(ctx, reinterpret_cast<qdc::cx*>(state), qdc::to_mat<2>(gate),
                             (uint32_t)pos, (uint32_t)pos, (uint32_t)n, "q1gate");
}

__attribute__((visibility("default"))) const char* q1gate_inv(qdc_complex* state,
                                                              const qdc_complex* gate,
                                                              size_t pos, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  if (pos >= n) return qdc::fail("pos is out of the bound.");
  qdc::mat<2> inv;
  QDC_TRY(qdc::inverse<2>(qdc::to_mat<2>(gate), inv));
  return qdc::apply_dense<2>(ctx, reinterpret_cast<qdc::cx*>(state), inv, (uint32_t)pos,
                             (uint32_t)pos, (uint32_t)n, "q1gate");
}

__attribute__((visibility("default"))) const char* q2gate(qdc_complex* state,
                                                          const qdc_complex* gate, size_t pos2,
                                                          size_t pos1, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  return qdc::apply_dense<4>(ctx, reinterpret_cast<qdc::cx*>(state), qdc::to_mat<4>(gate),
                             (uint32_t)pos2, (uint32_t)pos1, (uint32_t)n, "q2gate");
}

__attribute__((visibility("default"))) const char* q2gate_inv(qdc_complex* state,
                                                              const qdc_complex* gate,
                                                              size_t pos2, size_t pos1,
                                                              size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  qdc::mat<4> inv;
  QDC_TRY(qdc::inverse<4>(qdc::to_mat<4>(gate), inv));
  return qdc::apply_dense<4>(ctx, reinterpret_cast<qdc::cx*>(state), inv, (uint32_t)pos2,
                             (uint32_t)pos1, (uint32_t)n, "q2gate");
}

__attribute__((visibility("default"))) const char* q2gate_diag(qdc_complex* state,
                                                               const qdc_complex* gate,
                                                               size_t pos2, size_t pos1,
                                                               size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  return qdc::apply_diag(ctx, reinterpret_cast<qdc::cx*>(state), qdc::to_diag(gate),
                         (uint32_t)pos2, (uint32_t)pos1, (uint32_t)n, "q2gate_diag");
}

__attribute__((visibility("default"))) const char* get_q1density(const qdc_complex* state,
                                                                 qdc_complex* density,
                                                                 size_t pos, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  if (pos >= n) return qdc::fail("pos is out of the bound.");
  QDC_TRY(qdc::density<2>(ctx, reinterpret_cast<const qdc::cx*>(state), (uint32_t)pos,
                          (uint32_t)pos, (uint32_t)n, ctx.results, 0, 0));
  return qdc::abi_finish_reduction(ctx, density, 4);
}

__attribute__((visibility("default"))) const char* get_q2density(const qdc_complex* state,
                                                                 qdc_complex* density,
                                                                 size_t pos2, size_t pos1,
                                                                 size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  QDC_TRY(qdc::density<4>(ctx, reinterpret_cast<const qdc::cx*>(state), (uint32_t)pos2,
                          (uint32_t)pos1, (uint32_t)n, ctx.results, 0, 0));
  return qdc::abi_finish_reduction(ctx, density, 16);
}

__attribute__((visibility("default"))) const char* q1grad(const qdc_complex* fwd,
                                                          const qdc_complex* bwd,
                                                          qdc_complex* grad, size_t pos,
                                                          size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  if (pos >= n) return qdc::fail("pos out of range.");
  QDC_TRY(qdc::grad_dense<2>(ctx, reinterpret_cast<const qdc::cx*>(fwd),
                             reinterpret_cast<const qdc::cx*>(bwd), (uint32_t)pos, (uint32_t)pos,
                             (uint32_t)n, ctx.results, 0, 0));
  return qdc::abi_finish_reduction(ctx, grad, 4);
}

__attribute__((visibility("default"))) const char* q2grad(const qdc_complex* fwd,
                                                          const qdc_complex* bwd,
                                                          qdc_complex* grad, size_t pos2,
                                                          size_t pos1, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  QDC_TRY(qdc::grad_dense<4>(ctx, reinterpret_cast<const qdc::cx*>(fwd),
                             reinterpret_cast<const qdc::cx*>(bwd), (uint32_t)pos2,
                             (uint32_t)pos1, (uint32_t)n, ctx.results, 0, 0));
  return qdc::abi_finish_reduction(ctx, grad, 16);
}

__attribute__((visibility("default"))) const char* q2grad_diag(const qdc_complex* fwd,
                                                               const qdc_complex* bwd,
                                                               qdc_complex* grad, size_t pos2,
                                                               size_t pos1, size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  QDC_TRY(check_q2(pos2, pos1, n));
  QDC_TRY(qdc::grad_diag(ctx, reinterpret_cast<const qdc::cx*>(fwd),
                         reinterpret_cast<const qdc::cx*>(bwd), (uint32_t)pos2, (uint32_t)pos1,
                         (uint32_t)n, ctx.results, 0, 0));
  return qdc::abi_finish_reduction(ctx, grad, 4);
}

__attribute__((visibility("default"))) void conj_and_double(const qdc_complex* src,
                                                             qdc_complex* dst, size_t n) {
  QDC_VOID(elementwise_impl<1>(src, dst, n));
}

__attribute__((visibility("default"))) void add(const qdc_complex* src, qdc_complex* dst,
                                                size_t n) {
  QDC_VOID(elementwise_impl<2>(src, dst, n));
}

__attribute__((visibility("default"))) void copy(const qdc_complex* src, qdc_complex* dst,
                                                 size_t n) {
  QDC_VOID(elementwise_impl<0>(src, dst, n));
}

// ---- extensions beyond the reference's 18 entry points (include/qdc/dense.h) ----------------

__attribute__((visibility("default"))) const char* qdc_qkgate(qdc_complex* state,
                                                              const qdc_complex* gate,
                                                              const size_t* pos, size_t k,
                                                              size_t n) {
  QDC_ABI_BEGIN
  QDC_TRY(qdc::check_n(n));
  if (k < 1 || k > (size_t)qdc::QK_MAX)
    return qdc::fail("k = %zu qubits is out of the supported range (1..%d).", k, qdc::QK_MAX);
  if (k > n) return qdc::fail("k = %zu exceeds qubits_number %zu.", k, n);
  for (size_t b = 0; b < k; ++b) {
    if (pos[b] >= n) return qdc::fail("pos is out of the bound.");
    for (size_t c = 0; c < b; ++c)
      if (pos[c] == pos[b]) return qdc::fail("positions must be different.");
  }
  static qdc::QkRing rings[qdc::ABI_MAX_DEVICES];  // guarded by the ABI mutex
  return qdc::apply_qk(ctx, reinterpret_cast<qdc::cx*>(state), gate, pos, (uint32_t)k,
                       (uint32_t)n, rings[ctx.device]);
}

__attribute__((visibility("default"))) const char* qdc_abi_sync(void) {
  QDC_ABI_BEGIN
  QDC_HIP(hipStreamSynchronize(ctx.stream));
  return nullptr;
}

__attribute__((visibility("default"))) const char* qdc_abi_profile(int on) {
  QDC_ABI_BEGIN
  if (on) {
    QDC_HIP(hipStreamSynchronize(ctx.stream));
    ctx.prof.reset();
  }
  ctx.prof.on = on != 0;
  return nullptr;
}

__attribute__((visibility("default"))) size_t qdc_abi_profile_collect(qdc_kernel_stat* out,
                                                                      size_t cap) {
  std::lock_guard<std::mutex> lock(qdc::abi_mutex());
  qdc::Ctx* c = nullptr;
  if (qdc::abi_ctx(c)) return 0;
  return qdc::prof_collect(*c, out, cap);
}

}  // extern "C"
