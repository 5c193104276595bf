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
#include "qdc_rq.hpp"
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
  // physical qubit swaps the pass applies on its way out (its store writes the permuted
  // layout; later ops' positions are already rewritten), in order
  std::vector<std::pair<uint32_t, uint32_t>> swaps;
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
  uint32_t tile2_chunks = TILE_CHUNKS_2;  // two-state tile (chunks per state)
  uint32_t tile1_chunks = TILE_CHUNKS_1;  // one-state tile
  // Gate-only passes may permute the qubits of their tile on the way out (register-resident
  // passes store through any layout): the qubits the next ops need first move to the low
  // physical positions 0..LV+2 that every tile holds, so later tiles are not spent on pinned
  // qubits no op of theirs needs.
  bool permute = false;
  // two-state gate passes run register-resident (k_rq: FMAX_GRAD_RQ Gamma accumulators)
  bool rq_grad = false;
  // ... and are capped by their Gamma STAGES (stages holding a variable gate: one accumulator
  // each), not by their variable gates: a brickwork stage holds up to three of them
  bool gamma_stage_cap = true;
  // low physical positions a permuting pass fills with the qubits the next ops need first
  // (>= NLOW; more makes the next tiles' contiguous runs longer)
  uint32_t perm_low = (uint32_t)LV + 3;
  // rank bits of a sharded circuit (permuting passes carry their permutation through remaps)
  uint32_t ng = 0;
  // Mirrored schedules: the forward is scheduled so that its passes, run in reverse, are the
  // backward's passes (qdc_circuit.hpp mirror_schedule): on the two-state tile, under the
  // ordering rules of both directions, no gate after a density within a pass, and the
  // backward's cap on Gamma stages (stages holding a variable gate).  The uncompute then applies
  // exactly the adjoints of the forward's stage matrices.
  bool mirror = false;
  // trailing one-qubit stages move to the pass of their qubit's next two-qubit gate
  // (defer_trailing_q1; QDC_DEFER_Q1)
  bool defer_q1 = true;
  // a forward pass holds gates or densities, not both (round 6; QDC_DENS_SPLIT): a pass with
  // densities cannot be register-resident, so a mixed pass ran its gates on the LDS kernel
  // (C2 n = 28: one pass of 5 gate stages + 11 densities, 2.66 ms); split, the gates run
  // register-resident and the densities join density-only passes (k_dens1)
  bool split_dens = true;

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
    // a mirrored forward keeps the backward's order relations too
    if (mirror && !backward)
      return order_class(ins[op.instr].kind, false, inex) | order_class(ins[op.instr].kind, true, inex);
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
  // The low physical positions every tile holds: amplitude bits 0..LV-1 and chunk bits 0..2.
  static constexpr uint32_t NLOW = (uint32_t)LV + 3;
  // Choose the pass's swaps: rank the tile's qubits by the first upcoming op (`rest` of this
  // segment, then plan[next..]) that uses them; the first NLOW move to the low positions.
  void permute_after(FusionItem& it, std::vector<qdc_plan_op>& plan,
                     const std::vector<uint32_t>& rest, size_t next) const {
    // the low positions to fill: at least NLOW, at most the pass's contiguous run
    const uint32_t nlow = std::max(NLOW, std::min(perm_low, (uint32_t)LV + it.lc));
    std::vector<uint8_t> in_tile(nl, 0);
    for (uint32_t p = 0; p < (uint32_t)LV + it.lc; ++p) in_tile[p] = 1;
    for (uint32_t r = 0; r < it.h; ++r) in_tile[LV + it.hb[r]] = 1;
    std::vector<uint32_t> want;
    std::vector<uint8_t> ranked(nl, 0);
    auto see = [&](const qdc_plan_op& op) {
      if (op.type != QDC_PLAN_OP) return;
      for (uint32_t p : {op.pos2, op.pos1})
        if (p < nl && in_tile[p] && !ranked[p] && want.size() < nlow) {
          ranked[p] = 1;
          want.push_back(p);
        }
    };
    for (uint32_t k : rest) see(plan[k]);
    for (size_t k = next; k < plan.size() && want.size() < nlow; ++k) {
      if (plan[k].type == QDC_PLAN_REMAP) break;
      see(plan[k]);
    }
    std::vector<uint32_t> free_low;  // low positions whose qubit is not wanted
    for (uint32_t p = 0; p < nlow; ++p)
      if (!ranked[p]) free_low.push_back(p);
    // (sharded: positions < LV, inside the 16-B chunk, keep their qubit — a remap exchanges
    // whole chunks, so a later remap's victim must never land there; the remap planner never
    // picks them and remaps keep them in place)
    size_t f = 0;
    for (uint32_t p : want) {
      if (p < nlow) continue;
      while (f < free_low.size() && ng > 0 && free_low[f] < (uint32_t)LV) ++f;
      if (f == free_low.size()) break;
      it.swaps.push_back({p, free_low[f++]});
    }
    if (it.swaps.empty()) return;
    auto moved = [&](uint32_t p) {
      for (const auto& sw : it.swaps) {
        if (p == sw.first) p = sw.second;
        else if (p == sw.second) p = sw.first;
      }
      return p;
    };
    for (uint32_t k : rest) {
      plan[k].pos2 = moved(plan[k].pos2);
      plan[k].pos1 = moved(plan[k].pos1);
    }
    // the rest of the plan: positions through the permutation; across a remap (sharded
    // circuits) the permutation is carried through it (relabel_remap)
    std::vector<uint32_t> pi(nl + ng);
    for (uint32_t p = 0; p < nl + ng; ++p) pi[p] = p < nl ? moved(p) : p;
    for (size_t k = next; k < plan.size(); ++k) {
      if (plan[k].type == QDC_PLAN_REMAP) {
        relabel_remap(plan[k], pi);
        continue;
      }
      if (plan[k].type != QDC_PLAN_OP) continue;
      plan[k].pos2 = pi[plan[k].pos2];
      plan[k].pos1 = pi[plan[k].pos1];
    }
  }
  // Sharded circuits (ng rank bits): the plan's positions assume the layout the remap planner
  // simulated; a permuting pass changes the actual one by a permutation pi of the n physical
  // positions (local to local, rank bits fixed at first).  A later remap must move the same
  // logical qubits to the rank bits, so its victims become sorted(pi(V)); afterwards the actual
  // layout differs from the planned one by pi' = M_{pi(V)} o pi o M_V^-1 (M_X: the layout
  // change of a remap with victims X, qdc_shard.hpp QubitMap::apply), which may also reorder
  // the rank bits — later remaps bring them back through the same formula.
  void remap_map(const uint32_t* v, std::vector<uint32_t>& m) const {
    const uint32_t L = nl, n = nl + ng;
    m.assign(n, 0);
    uint32_t c = 0;
    for (uint32_t p = 0; p < L; ++p) {
      bool vic = false;
      for (uint32_t j = 0; j < ng; ++j) vic = vic || v[j] == p;
      if (!vic) m[p] = c++;
    }
    for (uint32_t j = 0; j < ng; ++j) m[v[j]] = L + j;
    for (uint32_t i = 0; i < ng; ++i) m[L + i] = L - ng + i;
  }
  void relabel_remap(qdc_plan_op& r, std::vector<uint32_t>& pi) const {
    uint32_t nv[8];
    for (uint32_t j = 0; j < ng; ++j) nv[j] = pi[r.victims[j]];
    std::sort(nv, nv + ng);
    std::vector<uint32_t> mv, mn, mvi(nl + ng), out(nl + ng);
    remap_map(r.victims, mv);
    remap_map(nv, mn);
    for (uint32_t p = 0; p < nl + ng; ++p) mvi[mv[p]] = p;
    for (uint32_t x = 0; x < nl + ng; ++x) out[x] = mn[pi[mvi[x]]];
    pi.swap(out);
    r.pack = 0;
    for (uint32_t j = 0; j < ng; ++j) {
      r.victims[j] = nv[j];
      r.pack |= (nv[j] != nl - ng + j) ? 1 : 0;
    }
  }

  // With `permute`, a fused gate-only pass gets `swaps` and the positions of every later op of
  // `plan` are rewritten to the permuted layout.
  std::vector<FusionItem> fuse_items(std::vector<qdc_plan_op>& plan, bool backward,
                                     size_t first_inject = SIZE_MAX) const {
    std::vector<FusionItem> items;
    const bool mfwd = mirror && !backward;  // a mirrored forward (see `mirror`)
    const uint32_t T = log2_of((backward || mfwd) ? tile2_chunks : tile1_chunks);
    const bool on = fuse && fuse_max_ops >= 2;
    // a mirrored forward's passes do not straddle the last differentiable density: the
    // backward's passes before its first injection are one-state (no cotangent yet)
    size_t msplit = SIZE_MAX;
    if (mfwd)
      for (size_t k = plan.size(); k-- > 0;)
        if (plan[k].type == QDC_PLAN_OP && is_meas(plan[k]) &&
            (ins[plan[k].instr].kind == QDC_DIFF_Q1_DENSITY ||
             ins[plan[k].instr].kind == QDC_DIFF_Q2_DENSITY)) {
          msplit = k + 1;
          break;
        }
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
             !(backward && j == first_inject && j > i) && !(j == msplit && j > i))
        ++j;
      // (a mirrored forward's passes are capped as the backward's two-state passes)
      const bool two = (backward && i >= first_inject) || mfwd;
      const bool gstage = two && rq_grad && gamma_stage_cap;
      const uint32_t gmax = gstage ? fuse_max_ops
                            : (two && rq_grad) ? (uint32_t)FMAX_GRAD_RQ : (uint32_t)FMAX_GRAD;
      std::vector<uint32_t> rem;
      for (size_t k = i; k < j; ++k) rem.push_back((uint32_t)k);
      while (!rem.empty()) {
        uint64_t mask = 0, blocked = 0;
        uint32_t nred = 0;
        uint32_t ndens = 0;  // a mirrored forward's densities (its reduction slots)
        uint32_t left = 0;  // order classes of the ops left for a later pass
        std::vector<uint32_t> pass, rest;
        int kind = -1;  // reverse sweep: a pass is injections only or gates only
        for (uint32_t k : rem) {
          const qdc_plan_op& g = plan[k];
          const uint64_t q = (1ull << g.pos2) | (1ull << g.pos1);
          const bool meas = is_meas(g);
          const uint32_t cls = op_class(g, backward);
          // (a mirrored forward: variable gates count toward the backward's Gamma cap,
          // densities toward the forward's reduction slots)
          const uint32_t isred = mfwd ? (is_var(ins[g.instr].kind) ? 1u : 0u)
                                 : ((!backward && meas) || (two && is_var(ins[g.instr].kind))) ? 1u : 0u;
          // reverse sweep: a pass is injections only or gates only; a mirrored forward's pass
          // is gates then densities (no gate after a density: its backward splits into the
          // injections, then the gates' mirrored stages)
          if ((backward && kind >= 0 && (int)meas != kind) || (mfwd && kind == 1 && !meas) ||
              (!backward && split_dens && kind == 0 && meas) ||
              (q & blocked) ||
              (mfwd && meas && ndens + 1 > (uint32_t)FMAX_GRAD) ||
              (conflicts_of(cls) & left) || pass.size() >= fuse_max_ops ||
              nred + isred > gmax || !tile_fits(mask | op_bits(g), T)) {
            blocked |= q;
            left |= cls;
            rest.push_back(k);
            continue;
          }
          pass.push_back(k);
          mask |= op_bits(g);
          nred += isred;
          ndens += (mfwd && meas) ? 1u : 0u;
          kind = (int)meas;
        }
        // Gamma-stage cap: drop gates from the end of the pass (in pass order no kept gate
        // depends on a dropped one) until its Gamma stages fit the accumulators
        if (gstage && nred > (uint32_t)FMAX_GRAD_RQ) {
          bool cut = false;
          while (pass.size() > 1 && gamma_stages(pass, plan, !mfwd) > (uint32_t)FMAX_GRAD_RQ) {
            rest.push_back(pass.back());
            pass.pop_back();
            cut = true;
          }
          if (cut) {
            std::sort(rest.begin(), rest.end());
            mask = 0;
            for (uint32_t k : pass) mask |= op_bits(plan[k]);
          }
        }
        if (defer_q1 && defer_trailing_q1(pass, rest, plan, backward)) {
          mask = 0;
          for (uint32_t k : pass) mask |= op_bits(plan[k]);
        }
        if (pass.size() == 1) {
          items.push_back(FusionItem{0, pass});
        } else {
          FusionItem it{2, pass};
          tile_config(mask, T, it.lc, it.h, it.hb);
          bool gates_only = it.lc >= NLOW - LV;  // the low positions are tile bits
          for (uint32_t k : pass) gates_only = gates_only && is_gate_op(plan[k]);
          if (permute && gates_only) permute_after(it, plan, rest, j);
          items.push_back(it);
        }
        rem.swap(rest);
      }
      i = j;
    }
    return items;
  }

  // A stage of one-qubit gates that ends its qubit's run in a pass, when that qubit's next op
  // (left for a later pass) is a two-qubit gate, moves to the later pass: there it joins the
  // two-qubit gate's stage instead of costing a stage of its own (2 complex MACs per amplitude
  // forward, 6 in the reverse sweep).  Only stages no later op of the pass depends on (shared
  // qubit or conflicting order classes) move; at least one stage stays.  Returns whether any
  // moved (rest stays in plan order).
  bool defer_trailing_q1(std::vector<uint32_t>& pass, std::vector<uint32_t>& rest,
                         const std::vector<qdc_plan_op>& plan, bool backward) const {
    if (pass.size() < 2 || rest.empty()) return false;
    const std::vector<std::vector<uint32_t>> sts = stage_partition(pass, plan, backward);
    if (sts.size() < 2) return false;
    std::vector<uint32_t> moved;
    size_t kept_stages = sts.size();
    for (const auto& st : sts) {
      if (kept_stages <= 1) break;
      // (one-qubit gates on one qubit only)
      bool q1only = true;
      for (uint32_t k : st)
        q1only = q1only && is_gate_op(plan[k]) && plan[k].pos2 == plan[k].pos1 &&
                 plan[k].pos2 == plan[st[0]].pos2;
      if (!q1only) continue;
      const uint32_t qb = plan[st[0]].pos2;
      const uint64_t qm = 1ull << qb;
      bool free = true;  // no later op of the pass depends on the stage
      for (uint32_t x : st) {
        const uint32_t cx = op_class(plan[x], backward);
        for (uint32_t y : pass) {
          if (y <= x || std::find(st.begin(), st.end(), y) != st.end()) continue;
          if (std::find(moved.begin(), moved.end(), y) != moved.end()) continue;
          const uint64_t yq = (1ull << plan[y].pos2) | (1ull << plan[y].pos1);
          if ((yq & qm) || (conflicts_of(cx) & op_class(plan[y], backward))) free = false;
        }
      }
      if (!free) continue;
      // the qubit's next op in the rest of the window: a two-qubit gate
      const qdc_plan_op* next = nullptr;
      for (uint32_t k : rest)
        if (k > st.back() && (((1ull << plan[k].pos2) | (1ull << plan[k].pos1)) & qm)) {
          next = &plan[k];
          break;
        }
      if (!next || !is_gate_op(*next) || next->pos2 == next->pos1) continue;
      moved.insert(moved.end(), st.begin(), st.end());
      --kept_stages;
    }
    if (moved.empty()) return false;
    std::vector<uint32_t> keep;
    for (uint32_t k : pass)
      if (std::find(moved.begin(), moved.end(), k) == moved.end()) keep.push_back(k);
    pass.swap(keep);
    rest.insert(rest.end(), moved.begin(), moved.end());
    std::sort(rest.begin(), rest.end());
    return true;
  }

  uint32_t gamma_stages(const std::vector<uint32_t>& pass, const std::vector<qdc_plan_op>& plan,
                        bool backward = true) const {
    uint32_t n = 0;
    for (const auto& st : stage_partition(pass, plan, backward)) {
      bool var = false;
      for (uint32_t k : st) var = var || (plan[k].type == QDC_PLAN_OP && is_var(ins[plan[k].instr].kind));
      n += var ? 1u : 0u;
    }
    return n;
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

// ---- register layouts of a register-resident pass (qdc_rq.hpp) -----------------------------
// A stage of the pass, in tile bits: kind FK_Q1 (t1 == t2), FK_Q2 or FK_DIAG (t1 < t2); deps =
// the earlier stages of the pass it must follow (shared qubit or conflicting order classes).
struct RqStage {
  uint32_t kind, t1, t2;
  uint64_t deps = 0;
};
constexpr int RQ_SLOTS_MAX = 5;  // register slots of a layout: 4, or 5 (k_rw two-state f32)
struct RqLayout {
  uint32_t ns = 4;  // register slots (register index bits 0..ns-1)
  uint32_t slot[RQ_SLOTS_MAX] = {~0u, ~0u, ~0u, ~0u, ~0u};  // tile bit held by register slot s
  // thread bits: the tile bits not in a slot, ascending — or, with tfix, tfirst[0..2] first
  // (a permuting pass's store layout: the bits that land on chunk bits 0..2)
  bool tfix = false;
  uint32_t tfirst[3] = {0, 0, 0};
  static RqLayout empty(uint32_t ns) {
    RqLayout L;
    L.ns = ns;
    return L;
  }
  bool operator==(const RqLayout& o) const {
    if (ns != o.ns || tfix != o.tfix) return false;
    for (uint32_t s = 0; s < ns; ++s)
      if (slot[s] != o.slot[s]) return false;
    return !tfix || (tfirst[0] == o.tfirst[0] && tfirst[1] == o.tfirst[1] &&
                     tfirst[2] == o.tfirst[2]);
  }
  // the thread bits in order (k < T - ns)
  uint32_t threads(uint32_t T, uint32_t* out) const {
    uint32_t k = 0;
    if (tfix)
      for (int i = 0; i < 3; ++i) out[k++] = tfirst[i];
    for (uint32_t q = 0; q < T && k < 8; ++q) {
      if (holds(q)) continue;
      if (tfix && (q == tfirst[0] || q == tfirst[1] || q == tfirst[2])) continue;
      out[k++] = q;
    }
    return k;
  }
  int find(uint32_t q) const {
    for (uint32_t s = 0; s < ns; ++s)
      if (slot[s] == q) return (int)s;
    return -1;
  }
  bool holds(uint32_t q) const { return find(q) >= 0; }
  // HBM layouts (load / store), lanes 0..7 reading 128 contiguous bytes: f32 (LV = 1) slot 0 =
  // tile bit 0 (a 16-B chunk is one thread's register pair) and tile bits 1..3 are thread bits
  // 0..2; f64 (LV = 0, a chunk is one amplitude) tile bits 0..2 are thread bits 0..2
  bool hbm_ok() const {
    if (LV == 0) return !holds(0) && !holds(1) && !holds(2);
    return slot[0] == 0 && !holds(1) && !holds(2) && !holds(3);
  }
};
// One step of a planned pass: a relayout to L, or stage `stage` run with slot case `cs`
// (qdc_rq.hpp: S1 * 8 + S2 for two-qubit / diagonal stages, the slot for one-qubit ones).
struct RqStep {
  bool relayout;
  RqLayout L;
  uint32_t stage, cs;
};
struct RqPlan {
  RqLayout load, store;
  std::vector<RqStep> steps;
};

// LDS index swizzle of the register-resident passes' relayouts.  A relayout writes (and reads)
// register j of lane l at index tp(l) ^ rp[j]: a 32-lane half of a ds_write/read_b64 is
// conflict-free when the images of lane bits 0..4 are independent mod 32 (64 banks of 4 B).
// The lane bits are the layout's five lowest thread bits — any tile bits — so f32 index bits
// 5..10 are XORed into bits 0..4 by the rows of RQ_SWZ, found by a search over the relayouts
// of the C2 step's 123 specialized passes (average bank multiplicity per half 2.06 -> 1.20;
// on a deep random circuit's 93 passes 2.28 -> 1.27; the k_fused swizzle swz, whose bits 9..10
// map to nothing, gave 2.06).  XOR-linear, so addresses stay tp ^ rp[j]; a bijection (the high
// bits are unchanged).  QDC_RQ_SWZ=0: swz.  f64 (16-B entries, other bank grouping): swz.
inline bool rq_swz_on() {
  static const bool on = [] {
    const char* e = getenv("QDC_RQ_SWZ");
    return !(e && atoi(e) == 0);
  }();
  return on;
}
inline uint32_t rq_swz(uint32_t i) {
  if (LV == 0 || !rq_swz_on()) return swz(i);
  constexpr uint32_t M[6] = {27u, 13u, 28u, 21u, 27u, 22u};
  uint32_t x = i;
  for (uint32_t b = 0; b < 6; ++b)
    if ((i >> (5 + b)) & 1u) x ^= M[b];
  return x;
}

// The layout's LDS descriptor (qdc_rq.hpp rq_layout): rp[j] = rq_swz(dep(j -> slots)),
// tv[k] = rq_swz(1 << k-th thread bit), thread bits = tile bits not in a slot, ascending.
inline rq_layout rq_descriptor(const RqLayout& L, uint32_t T) {
  rq_layout d{};
  for (uint32_t j = 0; j < (1u << L.ns); ++j) {
    uint32_t idx = 0;
    for (uint32_t s = 0; s < L.ns; ++s)
      if ((j >> s) & 1u) idx |= 1u << L.slot[s];
    d.rp[j] = rq_swz(idx);
  }
  uint32_t th[8];
  const uint32_t nt = L.threads(T, th);
  for (uint32_t k = 0; k < nt; ++k) d.tv[k] = rq_swz(1u << th[k]);
  return d;
}
// The HBM side of a load / store layout (rqio halves): chunk offsets of the thread bits and of
// the register chunk index (slots 1..3), with tile chunk bit c at global chunk bit
// c (c < lc) or hb[c - lc].
// dest (store of a permuting pass): tile bit q's value goes where tile bit dest[q] sits.
// f32: register chunk i = register pair (2i, 2i + 1), its index bits slots 1..3; f64: register
// chunk j = register j, index bits slots 0..3.
inline void rq_hbm(const RqLayout& L, uint32_t T, uint32_t lc, const uint32_t* hb,
                   uint64_t* gv, uint64_t* offi, const uint32_t* dest = nullptr) {
  auto gbit = [&](uint32_t tile_bit) -> uint64_t {  // tile bit >= LV -> global chunk offset
    const uint32_t c = (dest ? dest[tile_bit] : tile_bit) - (uint32_t)LV;
    return 1ull << (c < lc ? c : hb[c - lc]);
  };
  uint32_t th[8];
  const uint32_t nt = L.threads(T, th);
  uint32_t k = 0;
  for (; k < nt; ++k) gv[k] = gbit(th[k]);
  for (; k < 8; ++k) gv[k] = 0;
  constexpr uint32_t S0 = LV;  // the first slot that is a chunk bit
  for (uint32_t i = 0; i < ((1u << L.ns) >> LV); ++i) {
    uint64_t o = 0;
    for (uint32_t s = S0; s < L.ns; ++s)
      if ((i >> (s - S0)) & 1u) o += gbit(L.slot[s]);
    offi[i] = o;
  }
}

// Schedule a pass's stages on register layouts (T tile bits).  List scheduling: among the
// stages whose dependencies are done, run (lowest index first) one whose qubits sit in
// register slots; when none does, relayout.  A relayout's qubit set is a cover: the 4 qubits
// of a ready seed stage plus those of the stages that then become runnable, greedily in index
// order, filled with the qubits of the next stages.  Every ready stage is tried as the seed and
// the cover that runs the most stages before the next relayout wins (max closure; with
// max_closure = false, the lowest ready seed).  A last relayout whose cover runs every
// remaining stage is made an HBM layout if it can be, which saves the store's relayout
// (C2 n=28: 507 -> 497 relayouts per step, +1 % gates/s; random passes -8..16 %).  The pass starts in a load
// layout chosen the same way under the HBM constraint, and ends in an HBM-valid layout — for
// a permuting pass (src != nullptr: src[b] = the tile bit whose value lands on tile bit b,
// b < 4) the layout with slot 0 = src[0] and thread bits 0..2 = src[1..3].
// keep: every relayout keeps one register slot's tile bit in place (a cover includes a qubit of
// the current slots), so it can run through half the LDS buffer (qdc_spec.hpp spec_xchg_half)
inline RqPlan rq_plan(const std::vector<RqStage>& st, uint32_t T,
                      const uint32_t* src = nullptr, bool max_closure = true, uint32_t ns = 4,
                      bool keep = false) {
  const size_t n = st.size();
  auto qset = [&](size_t j, uint32_t* q) -> int {
    q[0] = st[j].t1;
    q[1] = st[j].t2;
    return st[j].t1 == st[j].t2 ? 1 : 2;
  };
  auto fits = [&](const RqLayout& L, size_t j) {
    return L.holds(st[j].t1) && L.holds(st[j].t2);
  };
  auto hbm_allowed = [](uint32_t q) { return LV == 0 ? q > 2 : (q == 0 || q > 3); };
  // the qubit set of a relayout: stage j0 first, then greedily the stages that become ready
  auto cover = [&](uint64_t done, size_t j0, std::vector<uint32_t> S, bool hbm) {
    auto add = [&](size_t j) {
      uint32_t q[2];
      const int m = qset(j, q);
      std::vector<uint32_t> T2 = S;
      for (int i = 0; i < m; ++i) {
        if (hbm && !hbm_allowed(q[i])) return false;
        if (std::find(T2.begin(), T2.end(), q[i]) == T2.end()) T2.push_back(q[i]);
      }
      if (T2.size() > ns) return false;
      S = T2;
      return true;
    };
    uint64_t sim = done;
    if (j0 < n && add(j0)) sim |= 1ull << j0;
    for (bool progress = true; progress;) {
      progress = false;
      for (size_t c = 0; c < n && !progress; ++c) {
        if ((sim >> c) & 1ull) continue;
        if ((st[c].deps & ~sim) != 0) continue;
        if (add(c)) {
          sim |= 1ull << c;
          progress = true;
        }
      }
    }
    // fill: qubits of the next stages in index order, then the lowest allowed bits
    for (size_t c = 0; c < n && S.size() < ns; ++c) {
      if ((sim >> c) & 1ull) continue;
      uint32_t q[2];
      const int m = qset(c, q);
      for (int i = 0; i < m && S.size() < ns; ++i)
        if ((!hbm || hbm_allowed(q[i])) && std::find(S.begin(), S.end(), q[i]) == S.end())
          S.push_back(q[i]);
    }
    for (uint32_t q = T; q-- > 0 && S.size() < ns;)
      if ((!hbm || hbm_allowed(q)) && std::find(S.begin(), S.end(), q) == S.end()) S.push_back(q);
    return S;
  };
  // slots for a qubit set: members of `prev` keep their slot, slot 0 = bit 0 if `hbm` (f32)
  auto place = [&](const std::vector<uint32_t>& S, const RqLayout& prev, bool hbm) {
    RqLayout L = RqLayout::empty(ns);
    if (hbm && LV == 1) L.slot[0] = 0;
    for (uint32_t q : S) {
      if (L.holds(q)) continue;
      const int ps = prev.find(q);
      if (ps >= 0 && L.slot[ps] == ~0u) L.slot[ps] = q;
    }
    for (uint32_t q : S) {
      if (L.holds(q)) continue;
      for (uint32_t s = 0; s < ns; ++s)
        if (L.slot[s] == ~0u) {
          L.slot[s] = q;
          break;
        }
    }
    return L;
  };
  // stages that run on the qubit set S from `done` on, without another relayout
  auto closure = [&](uint64_t done0, const std::vector<uint32_t>& S) {
    uint32_t smask = 0;
    for (uint32_t q : S) smask |= 1u << q;
    uint64_t sim = done0;
    int cnt = 0;
    for (bool progress = true; progress;) {
      progress = false;
      for (size_t c = 0; c < n; ++c) {
        if (((sim >> c) & 1ull) || (st[c].deps & ~sim) != 0) continue;
        if (!((smask >> st[c].t1) & 1u) || !((smask >> st[c].t2) & 1u)) continue;
        sim |= 1ull << c;
        ++cnt;
        progress = true;
      }
    }
    return cnt;
  };
  auto ready = [&](uint64_t done0, size_t j) {
    return !((done0 >> j) & 1ull) && (st[j].deps & ~done0) == 0;
  };
  // Max closure: every ready stage seeds a cover; the one that runs the most stages before
  // the next relayout wins (ties: the lowest seed).  With `hbm` (the load layout, or a last
  // layout that is also the store) the seeds are the stages an HBM layout can hold.
  auto best_cover = [&](uint64_t done0, const std::vector<uint32_t>& base, bool hbm) {
    std::vector<uint32_t> best;
    int best_cnt = -1;
    for (size_t j = 0; j < n; ++j) {
      if (!ready(done0, j)) continue;
      if (hbm && !(hbm_allowed(st[j].t1) && hbm_allowed(st[j].t2))) continue;
      std::vector<uint32_t> S = cover(done0, j, base, hbm);
      if (!max_closure) return S;  // greedy: the lowest ready seed
      const int cnt = closure(done0, S);
      if (cnt > best_cnt) {
        best_cnt = cnt;
        best = std::move(S);
      }
    }
    if (best_cnt < 0) best = cover(done0, n, base, hbm);
    return best;
  };
  RqPlan P;
  uint64_t done = 0;
  {  // load layout
    const RqLayout none = RqLayout::empty(ns);
    P.load = place(best_cover(0, LV == 1 ? std::vector<uint32_t>{0u} : std::vector<uint32_t>{}, true),
                   none, true);
  }
  RqLayout cur = P.load;
  for (size_t left = n; left > 0;) {
    size_t pick = n;
    for (size_t j = 0; j < n && pick == n; ++j)
      if (ready(done, j) && fits(cur, j)) pick = j;
    if (pick == n) {
      // a cover that runs every remaining stage and is itself an HBM layout saves the
      // relayout back at the end (plain passes: a permuting pass stores through src)
      std::vector<uint32_t> S;
      bool hbm = false;
      if (!src && max_closure) {
        S = best_cover(done, LV == 1 ? std::vector<uint32_t>{0u} : std::vector<uint32_t>{}, true);
        hbm = closure(done, S) == (int)left;
      }
      if (hbm && keep) {  // the HBM cover must keep one of the current slots in place
        const RqLayout L = place(S, cur, true);
        bool kept = false;
        for (uint32_t q = 0; q < ns; ++q) kept = kept || (L.slot[q] == cur.slot[q] && cur.slot[q] != ~0u);
        hbm = kept;
      }
      if (!hbm && keep) {  // the best cover that contains one of the current slots' qubits
        // (f32: tile bit 0 stays in slot 0 when it is there, so the HBM store layout, which
        // needs it there, keeps that slot too)
        int best_cnt = -1;
        const bool pin0 = LV == 1 && cur.slot[0] == 0;
        for (uint32_t q = 0; q < ns; ++q) {
          if (cur.slot[q] == ~0u || (pin0 && q != 0)) continue;
          std::vector<uint32_t> Sq = best_cover(done, {cur.slot[q]}, false);
          const int cnt = closure(done, Sq);
          if (cnt > best_cnt) {
            best_cnt = cnt;
            S = std::move(Sq);
          }
        }
      } else if (!hbm) {
        S = best_cover(done, {}, false);
      }
      cur = place(S, cur, hbm);
      P.steps.push_back(RqStep{true, cur, 0, 0});
      for (size_t j = 0; j < n && pick == n; ++j)
        if (ready(done, j) && fits(cur, j)) pick = j;
    }
    const RqStage& s = st[pick];
    const uint32_t cs = s.kind == FK_Q1 ? (uint32_t)cur.find(s.t1)
                                        : (uint32_t)(cur.find(s.t1) * 8 + cur.find(s.t2));
    P.steps.push_back(RqStep{false, cur, (uint32_t)pick, cs});
    done |= 1ull << pick;
    --left;
  }
  if (src) {
    RqLayout L = RqLayout::empty(ns);
    L.slot[0] = src[0];
    L.tfix = true;
    for (int i = 0; i < 3; ++i) L.tfirst[i] = src[1 + i];
    auto taken = [&](uint32_t q) {
      for (int i = 0; i < 4; ++i)
        if (src[i] == q) return true;
      return L.holds(q);
    };
    for (uint32_t s = 1; s < ns; ++s)  // keep the current slots' qubits where possible
      if (cur.slot[s] != ~0u && !taken(cur.slot[s])) L.slot[s] = cur.slot[s];
    for (uint32_t s = 1; s < ns; ++s)
      for (uint32_t q = T; L.slot[s] == ~0u && q-- > 0;)
        if (!taken(q)) L.slot[s] = q;
    P.store = L;
    P.steps.push_back(RqStep{true, P.store, 0, 0});
  } else if (cur.hbm_ok()) {
    P.store = cur;
  } else {
    std::vector<uint32_t> S;
    if (LV == 1) S.push_back(0u);
    for (uint32_t s = 0; s < ns; ++s)
      if (hbm_allowed(cur.slot[s]) && (LV == 0 || cur.slot[s] != 0)) S.push_back(cur.slot[s]);
    for (uint32_t q = T; q-- > 0 && S.size() < ns;)
      if (hbm_allowed(q) && std::find(S.begin(), S.end(), q) == S.end()) S.push_back(q);
    P.store = place(S, cur, true);
    P.steps.push_back(RqStep{true, P.store, 0, 0});
  }
  return P;
}

}  // namespace qdc
