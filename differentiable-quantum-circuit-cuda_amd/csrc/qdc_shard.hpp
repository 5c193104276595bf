// qdc_shard.hpp — the state sharded by high qubit index across ranks.
//
// The reference is single-GPU; this is the build's one added strategy.
//   * G = 2^g ranks; global amplitude index = rank * 2^(n-g) + local index.  Physical qubit
//     positions 0..n-g-1 are local, n-g..n-1 are the rank bits ("global").
//   * A logical->physical qubit map is kept.  Every gate / density / cotangent injection needs
//     its qubits local; when one is global, a REMAP swaps all g global qubits with g local
//     "victim" qubits (never the qubits the op needs), chosen Belady-style as the qubits whose
//     next use lies farthest ahead.  One remap = [pack kernel when the victims are not already
//     the top local bits] + ONE all-to-all per state: each rank's shard splits into G
//     contiguous chunks (chunk j = victim bit pattern j), chunk j goes to rank j, and the chunk
//     received from rank s lands at position s, so the old rank bits become the top local
//     bits.  That uses all G-1 xGMI links at once.
//   * Densities and gradients are per-shard partial sums: one all-reduce per call.
//
// The planner is pure host logic (no GPU), exported as qdc_plan() so the CPU tests can execute
// its plans on numpy shards exchanged over gloo.
#pragma once

#include <algorithm>
#include <limits>
#include <vector>

#include "qdc/circuit.h"

namespace qdc {

struct QubitMap {
  uint32_t n = 0, g = 0;
  std::vector<uint32_t> phys;  // logical -> physical
  std::vector<uint32_t> logi;  // physical -> logical
  void identity(uint32_t n_, uint32_t g_) {
    n = n_;
    g = g_;
    phys.resize(n);
    logi.resize(n);
    for (uint32_t q = 0; q < n; ++q) phys[q] = logi[q] = q;
  }
  uint32_t nl() const { return n - g; }
  bool local(uint32_t q) const { return phys[q] < nl(); }
  // After a remap with (ascending) local victims: non-victim local positions compact to
  // 0..nl-g-1 in order, old rank bit i -> local nl-g+i, victim j -> rank bit j.
  void apply(const uint32_t* victims) {
    const uint32_t L = nl(), low = L - g;
    std::vector<uint32_t> np(n);
    uint32_t c = 0;
    for (uint32_t p = 0; p < L; ++p) {
      bool v = false;
      for (uint32_t j = 0; j < g; ++j) v |= victims[j] == p;
      if (!v) np[p] = c++;
    }
    for (uint32_t j = 0; j < g; ++j) np[victims[j]] = L + j;
    for (uint32_t i = 0; i < g; ++i) np[L + i] = low + i;
    for (uint32_t q = 0; q < n; ++q) phys[q] = np[phys[q]];
    for (uint32_t q = 0; q < n; ++q) logi[phys[q]] = q;
  }
  // The inverse of apply(victims): the layout before that remap (a mirrored reverse sweep
  // replays the forward's remaps backwards, qdc_circuit.hpp unremap).
  void unapply(const uint32_t* victims) {
    const uint32_t L = nl(), low = L - g;
    std::vector<uint32_t> np(n), inv(n);
    uint32_t c = 0;
    for (uint32_t p = 0; p < L; ++p) {
      bool v = false;
      for (uint32_t j = 0; j < g; ++j) v |= victims[j] == p;
      if (!v) np[p] = c++;
    }
    for (uint32_t j = 0; j < g; ++j) np[victims[j]] = L + j;
    for (uint32_t i = 0; i < g; ++i) np[L + i] = low + i;
    for (uint32_t p = 0; p < n; ++p) inv[np[p]] = p;
    for (uint32_t q = 0; q < n; ++q) phys[q] = inv[phys[q]];
    for (uint32_t q = 0; q < n; ++q) logi[phys[q]] = q;
  }
  // exchange the qubits at physical positions a and b (a permuting fused pass's store)
  void swap_phys(uint32_t a, uint32_t b) {
    const uint32_t la = logi[a], lb = logi[b];
    phys[la] = b;
    phys[lb] = a;
    logi[a] = lb;
    logi[b] = la;
  }
};

inline bool instr_is_q1(int kind) {
  return kind == QDC_CONST_Q1 || kind == QDC_CONST_Q1_NONU || kind == QDC_VAR_Q1 ||
         kind == QDC_VAR_Q1_NONU || kind == QDC_Q1_DENSITY || kind == QDC_DIFF_Q1_DENSITY;
}

struct PlanIn {
  int kind;
  uint32_t a, b;  // logical qubits (a only for one-qubit kinds)
};

// ---- order classes -------------------------------------------------------------------------
// Ops may run out of program order (remap planning here, pass scheduling in qdc_fusion.hpp)
// only as gates on disjoint qubits commute, with these extra constraints (an op may not pass a
// skipped op of a conflicting class):
//  * a density commutes with a gate on other qubits only if the gate is unitary to working
//    precision; a cotangent injection (reverse sweep) only with const non-NonU gates, for which
//    the pull-back B = U^T = conj(U^+) = conj(A) by construction:
//      MEAS (densities / injections) <-> SENS (forward: NonU or inexact gates; reverse: NonU
//      or variable gates);
//  * reverse sweep: swapping two gates leaves the other's gradient unchanged only if the moved
//    gate has B^T A = I, i.e. its uncompute A is the true inverse; the reference uncomputes
//    non-NonU kinds with U^+, so a gate whose matrix is not unitary ("inexact") keeps its
//    order relative to variable gates:  INEX <-> VAR.
enum : uint32_t { OC_MEAS = 1, OC_SENS = 2, OC_VAR = 4, OC_INEX = 8 };
inline bool kind_is_gate(int k) { return k >= QDC_CONST_Q2 && k <= QDC_VAR_Q1_NONU; }
inline bool kind_is_density(int k) { return k >= QDC_Q2_DENSITY && k <= QDC_DIFF_Q1_DENSITY; }
inline bool kind_is_var(int k) {
  return k == QDC_VAR_Q1 || k == QDC_VAR_Q1_NONU || k == QDC_VAR_Q2 || k == QDC_VAR_Q2_NONU ||
         k == QDC_VAR_Q2_DIAG;
}
inline bool kind_is_nonu(int k) {
  return k == QDC_CONST_Q1_NONU || k == QDC_VAR_Q1_NONU || k == QDC_CONST_Q2_NONU ||
         k == QDC_VAR_Q2_NONU;
}
// inexact: the gate's matrix is not unitary to working precision (per call)
inline uint32_t order_class(int kind, bool backward, bool inexact) {
  uint32_t c = 0;
  if (kind_is_density(kind)) c |= OC_MEAS;
  if (kind_is_gate(kind)) {
    const bool inex = inexact && !kind_is_nonu(kind);
    if (kind_is_nonu(kind) || (backward ? kind_is_var(kind) : inex)) c |= OC_SENS;
    if (backward && kind_is_var(kind)) c |= OC_VAR;
    if (backward && inex) c |= OC_INEX;
  }
  return c;
}
inline uint32_t order_conflicts(uint32_t c) {
  return ((c & OC_MEAS) ? OC_SENS : 0u) | ((c & OC_SENS) ? OC_MEAS : 0u) |
         ((c & OC_VAR) ? OC_INEX : 0u) | ((c & OC_INEX) ? OC_VAR : 0u);
}

// Plan one pass over `ops` (program execution order; `index[i]` = instruction index,
// inexact[index] optional).  Commutation-aware: every op that is ready (no skipped earlier op
// on its qubits or of a conflicting class) and has all qubits local runs, in program order;
// only when nothing else can run does a REMAP swap the g global qubits with g local victims.
// Victims: never physical position 0 (the in-chunk bit) nor a qubit of the first blocked op
// (so it runs next: progress), farthest first use among the remaining ops first (Belady);
// ties: highest position (the top local bits need no pack).  On a brickwork circuit the
// global qubits' light cone grows a couple of qubits per layer, so a remap buys many layers
// instead of one.  Emits QDC_PLAN_OP / QDC_PLAN_REMAP records; `map` is updated in place.
// both_dirs: a mirrored forward (its plan, run in reverse, is the reverse sweep's), so ops keep
// the order relations of both directions.
inline void plan_pass(const std::vector<PlanIn>& ops, const std::vector<int>& index,
                      QubitMap& map, std::vector<qdc_plan_op>& out, bool backward = false,
                      const std::vector<uint8_t>* inexact = nullptr, bool both_dirs = false) {
  const uint32_t g = map.g;
  auto qmask = [&](const PlanIn& op) {
    return (1ull << op.a) | (instr_is_q1(op.kind) ? 0ull : (1ull << op.b));
  };
  auto emit = [&](size_t i) {
    const PlanIn& op = ops[i];
    qdc_plan_op o{};
    o.type = QDC_PLAN_OP;
    o.instr = index[i];
    o.pos2 = map.phys[op.a];
    o.pos1 = instr_is_q1(op.kind) ? o.pos2 : map.phys[op.b];
    out.push_back(o);
  };
  std::vector<uint32_t> cls(ops.size());
  for (size_t i = 0; i < ops.size(); ++i) {
    const bool inex = inexact && (size_t)index[i] < inexact->size() && (*inexact)[index[i]];
    cls[i] = order_class(ops[i].kind, backward, inex);
    if (both_dirs) cls[i] |= order_class(ops[i].kind, !backward, inex);
  }
  std::vector<size_t> rem(ops.size());
  for (size_t i = 0; i < ops.size(); ++i) rem[i] = i;
  while (!rem.empty()) {
    uint64_t blocked = 0;
    uint32_t left = 0;
    std::vector<size_t> rest;
    for (size_t i : rem) {
      const PlanIn& op = ops[i];
      const uint64_t q = qmask(op);
      const bool local = map.local(op.a) && (instr_is_q1(op.kind) || map.local(op.b));
      if ((q & blocked) || (order_conflicts(cls[i]) & left) || !local) {
        blocked |= q;
        left |= cls[i];
        rest.push_back(i);
        continue;
      }
      emit(i);
    }
    rem.swap(rest);
    if (rem.empty()) break;
    // remap: the first remaining op is blocked only by a global qubit
    const PlanIn& first = ops[rem[0]];
    const uint64_t keep = qmask(first);
    std::vector<std::pair<size_t, uint32_t>> cand;
    for (uint32_t p = 1; p < map.nl(); ++p) {
      const uint32_t q = map.logi[p];
      if (keep >> q & 1ull) continue;
      size_t nxt = std::numeric_limits<size_t>::max();
      for (size_t k = 0; k < rem.size(); ++k)
        if (qmask(ops[rem[k]]) >> q & 1ull) {
          nxt = k;
          break;
        }
      cand.push_back({nxt, p});
    }
    std::sort(cand.begin(), cand.end(), [](auto& x, auto& y) {
      return x.first != y.first ? x.first > y.first : x.second > y.second;
    });
    qdc_plan_op r{};
    r.type = QDC_PLAN_REMAP;
    r.instr = -1;
    r.nvictims = g;
    for (uint32_t j = 0; j < g; ++j) r.victims[j] = cand[j].second;
    std::sort(r.victims, r.victims + g);
    r.pack = 0;
    for (uint32_t j = 0; j < g; ++j) r.pack |= (r.victims[j] != map.nl() - g + j);
    map.apply(r.victims);
    out.push_back(r);
  }
}

// Active instructions of a pass, in execution order.
//   mode RUN / FORWARD: gates + (all | Diff) densities, forward order;
//   mode BACKWARD: gates + Diff densities, reverse order.
template <class InstrT>
inline void active_ops(const std::vector<InstrT>& ins, int mode, std::vector<PlanIn>& ops,
                       std::vector<int>& index) {
  auto active = [&](int k) {
    if (k <= QDC_VAR_Q1_NONU) return true;  // gates
    if (k == QDC_DIFF_Q1_DENSITY || k == QDC_DIFF_Q2_DENSITY) return true;
    return mode == QDC_PLAN_RUN;
  };
  const size_t L = ins.size();
  for (size_t t = 0; t < L; ++t) {
    const size_t k = (mode == QDC_PLAN_BACKWARD) ? L - 1 - t : t;
    if (!active(ins[k].kind)) continue;
    ops.push_back({ins[k].kind, ins[k].a, ins[k].b});
    index.push_back((int)k);
  }
}

inline uint32_t log2_exact(size_t x) {
  uint32_t r = 0;
  while (((size_t)1 << r) < x) ++r;
  return ((size_t)1 << r) == x ? r : UINT32_MAX;
}

}  // namespace qdc
