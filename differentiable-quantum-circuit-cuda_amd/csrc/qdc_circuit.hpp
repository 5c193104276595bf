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
#include <vector>

#include "qdc/circuit.h"
#include "qdc_device.hpp"

namespace qdc {

struct Instr {
  int kind;
  uint32_t a;  // q1: pos; q2: pos2
  uint32_t b;  // q2: pos1
};

inline bool is_q1_gate(int k) {
  return k == QDC_CONST_Q1 || k == QDC_CONST_Q1_NONU || k == QDC_VAR_Q1 || k == QDC_VAR_Q1_NONU;
}
inline bool is_q2_dense(int k) {
  return k == QDC_CONST_Q2 || k == QDC_VAR_Q2 || k == QDC_CONST_Q2_NONU || k == QDC_VAR_Q2_NONU;
}
inline bool is_diag(int k) { return k == QDC_CONST_Q2_DIAG || k == QDC_VAR_Q2_DIAG; }
inline bool is_const(int k) {
  return k == QDC_CONST_Q1 || k == QDC_CONST_Q1_NONU || k == QDC_CONST_Q2 ||
         k == QDC_CONST_Q2_NONU || k == QDC_CONST_Q2_DIAG;
}
inline bool is_var(int k) {
  return k == QDC_VAR_Q1 || k == QDC_VAR_Q1_NONU || k == QDC_VAR_Q2 || k == QDC_VAR_Q2_NONU ||
         k == QDC_VAR_Q2_DIAG;
}
inline bool is_nonu(int k) {
  return k == QDC_CONST_Q1_NONU || k == QDC_VAR_Q1_NONU || k == QDC_CONST_Q2_NONU ||
         k == QDC_VAR_Q2_NONU;
}
inline bool is_density(int k) {
  return k == QDC_Q1_DENSITY || k == QDC_Q2_DENSITY || k == QDC_DIFF_Q1_DENSITY ||
         k == QDC_DIFF_Q2_DENSITY;
}
inline bool is_diff_density(int k) {
  return k == QDC_DIFF_Q1_DENSITY || k == QDC_DIFF_Q2_DENSITY;
}
inline bool is_q1_density(int k) { return k == QDC_Q1_DENSITY || k == QDC_DIFF_Q1_DENSITY; }
inline int gate_len(int k) { return is_q2_dense(k) ? 16 : 4; }

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

struct Circuit {
  uint32_t n = 0;
  Ctx ctx;
  cx* initial = nullptr;
  cx* state = nullptr;
  cx* bwd = nullptr;
  cx* dens_dev = nullptr;
  size_t dens_cap = 0;
  cx* grads_dev = nullptr;
  size_t grads_cap = 0;
  cx* host_out = nullptr;  // pinned
  size_t host_cap = 0;
  std::vector<Instr> ins;

  const char* init(uint32_t qubits) {
    n = qubits;
    int dev = 0;
    QDC_HIP(hipGetDevice(&dev));
    QDC_TRY(ctx.init(dev));
    const size_t bytes = ((size_t)1 << n) * sizeof(cx);
    QDC_HIP(hipMalloc(&initial, bytes));
    QDC_HIP(hipMalloc(&state, bytes));
    // QuantizedTensor::new_standard + clone (circuit.rs:96-102)
    QDC_TRY(set_standard(ctx, initial, n));
    QDC_TRY(elementwise<0>(ctx, initial, state, n));
    QDC_HIP(hipStreamSynchronize(ctx.stream));
    return nullptr;
  }
  void destroy() {
    if (ctx.stream) (void)hipStreamSynchronize(ctx.stream);
    for (cx* p : {initial, state, bwd, dens_dev, grads_dev})
      if (p) (void)hipFree(p);
    if (host_out) (void)hipHostFree(host_out);
    ctx.destroy();
  }

  const char* ensure_dev(cx*& p, size_t& cap, size_t count) {
    if (count <= cap) return nullptr;
    if (p) {
      QDC_HIP(hipStreamSynchronize(ctx.stream));
      QDC_HIP(hipFree(p));
    }
    p = nullptr;
    QDC_HIP(hipMalloc(&p, sizeof(cx) * count));
    cap = count;
    return nullptr;
  }
  const char* ensure_host(size_t count) {
    if (count <= host_cap) return nullptr;
    if (host_out) {
      QDC_HIP(hipStreamSynchronize(ctx.stream));
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

  // --- forward (Circuit::run / Circuit::forward) --------------------------------------
  // Validation reproduces the reference's panic order: per instruction, pop then the
  // apply-time assertions; leftovers at the end (circuit.rs:170-211, 221-263).
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

  const char* apply_forward(const Instr& in, const qdc_complex* g, cx* s) {
    if (is_q1_gate(in.kind)) return apply_dense<2>(ctx, s, to_mat<2>(g), in.a, in.a, n, "apply_q1");
    if (is_q2_dense(in.kind))
      return apply_dense<4>(ctx, s, to_mat<4>(g), in.a, in.b, n, "apply_q2");
    return apply_diag(ctx, s, to_diag(g), in.a, in.b, n, "apply_q2_diag");
  }

  const char* execute(int mode, const Flat& cg, const Flat& vg, qdc_complex* out) {
    std::vector<size_t> gidx;
    QDC_TRY(validate_forward(cg, vg, gidx));
    const size_t nout = output_count(mode);
    QDC_TRY(ensure_dev(dens_dev, dens_cap, std::max<size_t>(nout, 1) * RED));
    QDC_TRY(elementwise<0>(ctx, initial, state, n));  // data_transfer (quantized_tensor.rs:169-176)
    uint32_t o = 0;
    for (size_t k = 0; k < ins.size(); ++k) {
      const Instr& in = ins[k];
      if (is_const(in.kind)) {
        QDC_TRY(apply_forward(in, cg.at(gidx[k]), state));
      } else if (is_var(in.kind)) {
        QDC_TRY(apply_forward(in, vg.at(gidx[k]), state));
      } else if (is_diff_density(in.kind) || mode == QDC_MODE_RUN) {
        if (is_q1_density(in.kind))
          QDC_TRY(density<2>(ctx, state, in.a, in.a, n, dens_dev, o++, 0));
        else
          QDC_TRY(density<4>(ctx, state, in.a, in.b, n, dens_dev, o++, 0));
      }
    }
    QDC_TRY(ctx.flush());
    return collect(dens_dev, nout, out, [&](size_t j) {
      size_t c = 0;
      for (auto& in : ins)
        if (is_diff_density(in.kind) || (mode == QDC_MODE_RUN && is_density(in.kind))) {
          if (c == j) return is_q1_density(in.kind) ? 4 : 16;
          ++c;
        }
      return 0;
    });
  }

  template <class F>
  const char* collect(const cx* dev, size_t count, qdc_complex* out, F width_of) {
    if (count == 0) {
      QDC_HIP(hipStreamSynchronize(ctx.stream));
      return nullptr;
    }
    QDC_TRY(ensure_host(count * RED));
    QDC_HIP(hipMemcpyAsync(host_out, dev, sizeof(cx) * count * RED, hipMemcpyDeviceToHost,
                           ctx.stream));
    QDC_HIP(hipStreamSynchronize(ctx.stream));
    // widths are computed once, in order
    size_t w = 0;
    std::vector<int> widths(count);
    for (size_t j = 0; j < count; ++j) widths[j] = width_of(j);
    for (size_t j = 0; j < count; ++j) {
      for (int k = 0; k < widths[j]; ++k) {
        out[w + k].re = host_out[j * RED + k].x;
        out[w + k].im = host_out[j * RED + k].y;
      }
      w += widths[j];
    }
    return nullptr;
  }

  // --- backward (Circuit::backward, circuit.rs:266-429) --------------------------------
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

  const char* backward(const Flat& dg, const Flat& cg, const Flat& vg, qdc_complex* out) {
    std::vector<size_t> gidx;
    QDC_TRY(validate_backward(dg, cg, vg, gidx));
    const size_t nvar = n_var();
    if (!bwd) QDC_HIP(hipMalloc(&bwd, ((size_t)1 << n) * sizeof(cx)));
    QDC_TRY(ensure_dev(grads_dev, grads_cap, std::max<size_t>(nvar, 1) * RED));
    // variable gates met before the first cotangent keep zero gradients (circuit.rs:327-331)
    QDC_HIP(hipMemsetAsync(grads_dev, 0, sizeof(cx) * std::max<size_t>(nvar, 1) * RED,
                           ctx.stream));
    cx* f = state;
    bool have_bwd = false;
    size_t var_no = nvar;  // forward index of the next variable gate met in reverse
    for (size_t kk = ins.size(); kk-- > 0;) {
      const Instr& in = ins[kk];
      if (is_const(in.kind) || is_var(in.kind)) {
        const bool var = is_var(in.kind);
        if (var) --var_no;
        const qdc_complex* g = var ? vg.at(gidx[kk]) : cg.at(gidx[kk]);
        cx* gbase = (var && have_bwd) ? grads_dev : nullptr;
        if (is_diag(in.kind)) {
          const diag4 d = to_diag(g);
          if (have_bwd)
            QDC_TRY(reverse_diag(ctx, f, bwd, d, in.a, in.b, n, gbase, (uint32_t)var_no));
          else
            QDC_TRY(apply_diag(ctx, f, conj_diag(d), in.a, in.b, n, "uncompute_q2_diag"));
        } else if (is_q1_gate(in.kind)) {
          const mat<2> u = to_mat<2>(g);
          mat<2> A;
          if (is_nonu(in.kind))
            QDC_TRY(inverse<2>(u, A));
          else
            A = conj_transpose<2>(u);
          if (have_bwd)
            QDC_TRY(reverse_dense<2>(ctx, f, bwd, A, transpose<2>(u), in.a, in.a, n, gbase,
                                     (uint32_t)var_no));
          else
            QDC_TRY(apply_dense<2>(ctx, f, A, in.a, in.a, n, "uncompute_q1"));
        } else {
          const mat<4> u = to_mat<4>(g);
          mat<4> A;
          if (is_nonu(in.kind))
            QDC_TRY(inverse<4>(u, A));
          else
            A = conj_transpose<4>(u);
          if (have_bwd)
            QDC_TRY(reverse_dense<4>(ctx, f, bwd, A, transpose<4>(u), in.a, in.b, n, gbase,
                                     (uint32_t)var_no));
          else
            QDC_TRY(apply_dense<4>(ctx, f, A, in.a, in.b, n, "uncompute_q2"));
        }
      } else if (is_diff_density(in.kind)) {
        const qdc_complex* gd = dg.at(gidx[kk]);
        if (is_q1_density(in.kind))
          QDC_TRY(inject<2>(ctx, f, bwd, transpose<2>(to_mat<2>(gd)), in.a, in.a, n, !have_bwd));
        else
          QDC_TRY(inject<4>(ctx, f, bwd, transpose<4>(to_mat<4>(gd)), in.a, in.b, n, !have_bwd));
        have_bwd = true;
      }
    }
    QDC_TRY(ctx.flush());
    std::vector<int> widths;
    for (auto& in : ins)
      if (is_var(in.kind)) widths.push_back(gate_len(in.kind));
    return collect(grads_dev, nvar, out, [&](size_t j) { return widths[j]; });
  }
};

}  // namespace qdc
