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
};

inline bool instr_is_q1(int kind) {
  return kind == QDC_CONST_Q1 || kind == QDC_CONST_Q1_NONU || kind == QDC_VAR_Q1 ||
         kind == QDC_VAR_Q1_NONU || kind == QDC_Q1_DENSITY || kind == QDC_DIFF_Q1_DENSITY;
}

struct PlanIn {
  int kind;
  uint32_t a, b;  // logical qubits (a only for one-qubit kinds)
};

// Plan one pass over `ops` (already in execution order; `index[i]` = instruction index).
// Emits QDC_PLAN_OP / QDC_PLAN_REMAP records; `map` is updated in place.
inline void plan_pass(const std::vector<PlanIn>& ops, const std::vector<int>& index,
                      QubitMap& map, std::vector<qdc_plan_op>& out) {
  const uint32_t g = map.g;
  const size_t L = ops.size();
  // next_use[i][q] is computed lazily by a forward scan at remap time (remaps are rare)
  auto uses = [&](size_t i, uint32_t q) {
    return ops[i].a == q || (!instr_is_q1(ops[i].kind) && ops[i].b == q);
  };
  for (size_t i = 0; i < L; ++i) {
    const PlanIn& op = ops[i];
    const bool q1 = instr_is_q1(op.kind);
    const bool need = g > 0 && (!map.local(op.a) || (!q1 && !map.local(op.b)));
    if (need) {
      // candidates: local physical positions >= 1 (never the in-chunk bit 0), not holding an
      // operand of this op; score = distance to the next use of the qubit they hold
      std::vector<std::pair<size_t, uint32_t>> cand;
      for (uint32_t p = 1; p < map.nl(); ++p) {
        const uint32_t q = map.logi[p];
        if (q == op.a || (!q1 && q == op.b)) continue;
        size_t nxt = std::numeric_limits<size_t>::max();
        for (size_t k = i + 1; k < L; ++k)
          if (uses(k, q)) {
            nxt = k;
            break;
          }
        cand.push_back({nxt, p});
      }
      // farthest next use first; ties: highest position (keeps the pack coalesced, and the top
      // local bits need no pack at all)
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
    qdc_plan_op o{};
    o.type = QDC_PLAN_OP;
    o.instr = index[i];
    o.pos2 = map.phys[op.a];
    o.pos1 = q1 ? o.pos2 : map.phys[op.b];
    out.push_back(o);
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
