// qdc.hip — the single translation unit of libqdc_{f32,f64}.so.
//
// Build (see Makefile): hipcc -O3 --offload-arch=gfx950 -fPIC -shared [-DQDC_F64]
// Exports: the 18 reference primitives (include/qdc/primitives.h) and the circuit runtime
// (include/qdc/circuit.h).  Everything else has hidden visibility.
#include "qdc_circuit.hpp"
#include "qdc_primitives.hpp"

struct qdc_circuit {
  qdc::Circuit impl;
};

#define QDC_API extern "C" __attribute__((visibility("default")))

QDC_API const char* qdc_circuit_new(qdc_circuit** out, size_t qubits_number) {
  *out = nullptr;
  QDC_TRY(qdc::check_n(qubits_number));
  qdc_circuit* c = new qdc_circuit();
  const char* e = c->impl.init((uint32_t)qubits_number);
  if (e) {
    c->impl.destroy();
    delete c;
    return e;
  }
  *out = c;
  return nullptr;
}

QDC_API void qdc_circuit_free(qdc_circuit* c) {
  if (!c) return;
  c->impl.destroy();
  delete c;
}

QDC_API size_t qdc_circuit_qubits(const qdc_circuit* c) { return c->impl.n; }

QDC_API const char* qdc_circuit_set_state_from_vector(qdc_circuit* c, const qdc_complex* vec,
                                                      size_t len) {
  // QuantizedTensor::set_from_host + get_qubits_number (quantized_tensor.rs:44-52, 76-80)
  if (len == 0 || (len & (len - 1)) != 0) return qdc::fail("State size is not a power of 2.");
  if (len != ((size_t)1 << c->impl.n))
    return qdc::fail("Size of the given state does not match the size of the tensor.");
  QDC_HIP(hipMemcpyAsync(c->impl.initial, vec, len * sizeof(qdc_complex), hipMemcpyHostToDevice,
                         c->impl.ctx.stream));
  QDC_HIP(hipStreamSynchronize(c->impl.ctx.stream));
  return nullptr;
}

QDC_API const char* qdc_circuit_push(qdc_circuit* c, int kind, size_t pos2, size_t pos1) {
  if (kind < QDC_CONST_Q2 || kind > QDC_DIFF_Q1_DENSITY)
    return qdc::fail("unknown instruction kind %d", kind);
  const bool q1 = qdc::is_q1_gate(kind) || qdc::is_q1_density(kind);
  c->impl.ins.push_back({kind, (uint32_t)pos2, q1 ? 0u : (uint32_t)pos1});
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
  qdc::Flat cf(cg, cl, nc), vf(vg, vl, nv);
  return c->impl.execute(mode, cf, vf, dens);
}

QDC_API const char* qdc_circuit_backward(qdc_circuit* c, const qdc_complex* dg, const size_t* dl,
                                         size_t nd, const qdc_complex* cg, const size_t* cl,
                                         size_t nc, const qdc_complex* vg, const size_t* vl,
                                         size_t nv, qdc_complex* grads) {
  qdc::Flat df(dg, dl, nd), cf(cg, cl, nc), vf(vg, vl, nv);
  return c->impl.backward(df, cf, vf, grads);
}

QDC_API const char* qdc_circuit_get_state(qdc_circuit* c, int which, qdc_complex* host,
                                          size_t len) {
  qdc::Circuit& k = c->impl;
  if (len != ((size_t)1 << k.n)) return qdc::fail("state length mismatch");
  const qdc::cx* src = which == 0 ? k.state : which == 1 ? k.initial : k.bwd;
  if (!src) return qdc::fail("state %d is not allocated", which);
  QDC_HIP(hipMemcpyAsync(host, src, len * sizeof(qdc_complex), hipMemcpyDeviceToHost,
                         k.ctx.stream));
  QDC_HIP(hipStreamSynchronize(k.ctx.stream));
  return nullptr;
}

QDC_API const char* qdc_circuit_sync(qdc_circuit* c) {
  QDC_HIP(hipStreamSynchronize(c->impl.ctx.stream));
  return nullptr;
}

QDC_API const char* qdc_circuit_profile(qdc_circuit* c, int on) {
  qdc::Ctx& x = c->impl.ctx;
  if (on) {
    QDC_HIP(hipStreamSynchronize(x.stream));
    x.prof.reset();
  }
  x.prof.on = on != 0;
  return nullptr;
}

QDC_API size_t qdc_circuit_profile_collect(qdc_circuit* c, qdc_kernel_stat* out, size_t cap) {
  qdc::Ctx& x = c->impl.ctx;
  (void)hipStreamSynchronize(x.stream);
  std::vector<qdc_kernel_stat> agg;
  for (auto& r : x.prof.recs) {
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
  }
  for (size_t i = 0; i < agg.size() && i < cap; ++i) out[i] = agg[i];
  return agg.size();
}

QDC_API const char* qdc_build_info(void) {
#ifdef QDC_F64
  return "qdc f64 gfx950";
#else
  return "qdc f32 gfx950";
#endif
}
