// qdc_fusion.hpp — host-side scheduling of fused passes: which gates,
// densities and cotangent injections share one HBM pass, the tile each pass uses, and how a
// pass splits into register stages.  Pure host code: the circuit runtime executes the result,
// and qdc_fusion_schedule (include/qdc/circuit.h) exposes it to CPU tests.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <vector>

#include "qdc/circuit.h"
#include "qdc_kernels.hpp"
#include "qdc_shard.hpp"

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

// One unit of work of a pass program: a single plan op (type 0), a remap (1) or a fused pass
// (2) with its tile: lc contiguous chunk bits + h row bits hb[].
struct FusionItem {
  int type;
  std::vector<uint32_t> ops;  // plan indices, in execution order for type 2 passes
  uint32_t lc = 0, h = 0, hb[FMAX_ROWS] = {};
};

struct FusionPlanner {
  static constexpr uint32_t TILE_CHUNKS_1 = 2048;  // one-state fused tile (chunks)
  static constexpr uint32_t TILE_CHUNKS_2 = 1024;  // two-state fused tile (chunks per state)
  const std::vector<Instr>& ins;
  const std::vector<uint8_t>& inexact;  // per instruction: gate matrix not unitary to precision
  uint32_t nl;                           // local qubits of a shard
  bool fuse;
  bool fuse_meas;
  uint32_t fuse_max_ops;
  uint32_t fuse_lcmin;

  static uint32_t log2_of(uint64_t x) {
    uint32_t k = 0;
    while ((1ull << k) < x) ++k;
    return k;
  }
  // ---- fusion: gates whose qubits fit one tile run as one HBM pass ---------------------------
  // Gates on disjoint qubits commute, so within a segment of consecutive gate ops (bounded by
  // remaps, densities and cotangent injections) a pass may take any gate none of whose
  // earlier same-qubit gates is left for a later pass.  Each pass is built greedily in
  // program order: a gate joins if it is ready and its qubits still fit the tile, otherwise
  // its qubits are blocked for the rest of the scan.  Per qubit, gates keep program order, so
  // the result equals the sequential one up to floating-point rounding.

  uint64_t chunk_bits_of(uint32_t p) const { return p >= (uint32_t)LV ? 1ull << (p - LV) : 0ull; }
  // A full tile of 2^T chunks: lc contiguous chunk bits (>= fuse_lcmin) plus h = T - lc row
  // bits that cover the group's far target bits, padded with the lowest free bits above lc.
  // States with fewer than 2^T chunks are not fused.
  bool tile_config(uint64_t mask, uint32_t T, uint32_t& lc, uint32_t& h, uint32_t* hb) const {
    const uint32_t cbits = nl - LV;
    if (cbits < T) return false;
    for (int l = (int)T; l >= (int)fuse_lcmin; --l) {
      uint32_t rows = 0, tmp[64];
      for (uint32_t c = (uint32_t)l; c < cbits; ++c)
        if (mask >> c & 1ull) tmp[rows++] = c;
      if (rows > (uint32_t)FMAX_ROWS || (uint32_t)l + rows > T) continue;
      for (uint32_t c = (uint32_t)l; c < cbits && (uint32_t)l + rows < T; ++c)
        if (!(mask >> c & 1ull)) tmp[rows++] = c;
      if ((uint32_t)l + rows != T || rows > (uint32_t)FMAX_ROWS) continue;
      std::sort(tmp, tmp + rows);
      lc = (uint32_t)l;
      h = rows;
      for (uint32_t k = 0; k < rows; ++k) hb[k] = tmp[k];
      return true;
    }
    return false;
  }
  bool tile_fits(uint64_t mask, uint32_t T) const {
    if (nl - LV < T) return false;
    for (int l = (int)T; l >= (int)fuse_lcmin; --l) {
      const uint32_t rows = (uint32_t)__builtin_popcountll(mask >> l);
      if (rows <= (uint32_t)FMAX_ROWS && (uint32_t)l + rows <= T) return true;
    }
    return false;
  }

  // Ordering rules beyond "same qubit => program order" (qdc_stage.hpp has the algebra):
  //  * a density commutes with unitary gates on other qubits, not with non-unitary ones;
  //  * a cotangent injection (reverse sweep) commutes only with const unitary gates on other
  //    qubits: a variable gate's gradient sees the bwd state, so it keeps its order.
  // "meas" ops (densities, injections) and "sensitive" gates (non-unitary; in the reverse
  // sweep also variable) therefore never pass each other: once one kind is left for a later
  // pass or stage, every later op of the other kind is too (order classes, below).
  bool is_meas(const qdc_plan_op& op) const {
    return op.type == QDC_PLAN_OP && is_density(ins[op.instr].kind);
  }
  // order classes (qdc_shard.hpp): an op may not pass a skipped op of a conflicting class
  uint32_t op_class(const qdc_plan_op& op, bool backward) const {
    if (op.type != QDC_PLAN_OP) return 0;
    const bool inex = op.instr < inexact.size() && inexact[op.instr];
    return order_class(ins[op.instr].kind, backward, inex);
  }
  static uint32_t conflicts_of(uint32_t c) { return order_conflicts(c); }
  bool is_gate_op(const qdc_plan_op& op) const {
    if (op.type != QDC_PLAN_OP) return false;
    const int k = ins[op.instr].kind;
    return is_const(k) || is_var(k);
  }
  uint64_t op_bits(const qdc_plan_op& op) const {
    return chunk_bits_of(op.pos2) | chunk_bits_of(op.pos1);
  }

  // backward: plan indices >= first_inject run two-state (bwd exists); a pass never spans it.
  std::vector<FusionItem> fuse_items(const std::vector<qdc_plan_op>& plan, bool backward,
                               size_t first_inject = SIZE_MAX) const {
    std::vector<FusionItem> items;
    const uint32_t T = log2_of(backward ? TILE_CHUNKS_2 : TILE_CHUNKS_1);
    const bool on = fuse && fuse_max_ops >= 2;
    auto fusable = [&](size_t k) {
      const qdc_plan_op& op = plan[k];
      if (!(is_gate_op(op) || (fuse_meas && is_meas(op))) || !tile_fits(op_bits(op), T))
        return false;
      // injections need bwd: only in the two-state part
      return !(backward && is_meas(op) && k < first_inject);
    };
    size_t i = 0;
    while (i < plan.size()) {
      const qdc_plan_op& op = plan[i];
      if (op.type == QDC_PLAN_REMAP) {
        items.push_back(FusionItem{1, {(uint32_t)i}});
        ++i;
        continue;
      }
      if (!on || !fusable(i)) {
        items.push_back(FusionItem{0, {(uint32_t)i}});
        ++i;
        continue;
      }
      size_t j = i;
      while (j < plan.size() && plan[j].type == QDC_PLAN_OP && fusable(j) &&
             !(backward && j == first_inject && j > i))
        ++j;
      const bool two = backward && i >= first_inject;
      std::vector<uint32_t> rem;
      for (size_t k = i; k < j; ++k) rem.push_back((uint32_t)k);
      while (!rem.empty()) {
        uint64_t mask = 0, blocked = 0;
        uint32_t nred = 0;
        uint32_t left = 0;  // order classes of the ops left for a later pass
        std::vector<uint32_t> pass, rest;
        int kind = -1;  // reverse sweep: a pass is injections only or gates only
        for (uint32_t k : rem) {
          const qdc_plan_op& g = plan[k];
          const uint64_t q = (1ull << g.pos2) | (1ull << g.pos1);
          const bool meas = is_meas(g);
          const uint32_t cls = op_class(g, backward);
          const uint32_t isred =
              ((!backward && meas) || (two && is_var(ins[g.instr].kind))) ? 1u : 0u;
          if ((backward && kind >= 0 && (int)meas != kind) || (q & blocked) ||
              (conflicts_of(cls) & left) || pass.size() >= fuse_max_ops ||
              nred + isred > (uint32_t)FMAX_GRAD || !tile_fits(mask | op_bits(g), T)) {
            blocked |= q;
            left |= cls;
            rest.push_back(k);
            continue;
          }
          pass.push_back(k);
          mask |= op_bits(g);
          nred += isred;
          kind = (int)meas;
        }
        if (pass.size() == 1) {
          items.push_back(FusionItem{0, pass});
        } else {
          FusionItem it{2, pass};
          tile_config(mask, T, it.lc, it.h, it.hb);
          items.push_back(it);
        }
        rem.swap(rest);
      }
      i = j;
    }
    return items;
  }

  // Split a pass (plan indices in pass order) into stages: greedy in program order, a gate
  // joins the current stage if none of its qubits is blocked (an earlier gate on it is left
  // for a later stage) and the stage stays within two qubits.  Per qubit, order is kept.
  std::vector<std::vector<uint32_t>> stage_partition(const std::vector<uint32_t>& pass,
                                                     const std::vector<qdc_plan_op>& plan,
                                                     bool backward) const {
    std::vector<std::vector<uint32_t>> stages;
    std::vector<uint32_t> rem = pass;
    while (!rem.empty()) {
      std::vector<uint32_t> st, rest;
      uint64_t q = 0, blocked = 0;
      uint32_t left = 0;
      bool closed = false;
      for (uint32_t k : rem) {
        if (closed) {
          rest.push_back(k);
          continue;
        }
        const qdc_plan_op& g = plan[k];
        const uint64_t gq = (1ull << g.pos2) | (1ull << g.pos1);
        const bool meas = is_meas(g);
        const uint32_t cls = op_class(g, backward);
        bool bad = (gq & blocked) || (conflicts_of(cls) & left);
        if (!bad && meas) {
          if (st.empty()) {  // a density / injection is a stage of its own
            st.push_back(k);
            closed = true;
            continue;
          }
          bad = true;
        }
        if (!bad && __builtin_popcountll(q | gq) > 2) bad = true;
        if (bad) {
          blocked |= gq;
          left |= cls;
          rest.push_back(k);
          continue;
        }
        st.push_back(k);
        q |= gq;
      }
      stages.push_back(std::move(st));
      rem.swap(rest);
    }
    return stages;
  }

};

}  // namespace qdc
