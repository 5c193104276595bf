// qdc_stage.hpp — host algebra of the fused passes' register stages.
//
// A fused pass is split into stages: runs of gates (per-qubit program order kept) whose
// qubits all lie in one pair {lo, hi} of tile bits (or one bit).  The kernel treats a stage as
// one virtual gate: it applies the stage products A = A_m ... A_1 and B = B_m ... B_1 and, for
// the reverse sweep, accumulates ONE outer product Gamma = sum b0 f0^T of the stage-entry
// states (instead of one per gate).  Every gate's gradient follows exactly (linear algebra):
//
//   gate j of the stage, processed after j-1 others:
//     f_j = A_j ... A_1 f0,   b_{j-1} = B_{j-1} ... B_1 b0
//     G_j = sum b_{j-1} f_j^T = (B_{j-1} ... B_1) Gamma (A_j ... A_1)^T      (stage basis)
//   then a partial trace over the stage qubits the gate does not touch, in the gate's own
//   (pos2, pos1) index order — the quantity the reference accumulates per gate
//   (get_q{1,2}_grad, circuit.rs:320-392; primitives.cu:202-354).
//
// Stage basis: index r = 2*bit(hi) + bit(lo) (a one-qubit stage: r = bit).  Products are
// formed on the host in a wider type than the state's (f32 states: double; f64 states: x87
// long double, 64-bit significand) and rounded once to the state precision for the device: a
// stage matrix then differs from the exact product of its gates by half an ulp of the state
// precision, as a single gate's matrix does, instead of by the rounding of every product step.
#pragma once

#include <complex>
#include <vector>

namespace qdc {

#ifdef QDC_F64
using hreal = long double;
#else
using hreal = double;
#endif

template <class T>
struct SMatT {  // R x R, row-major, R = 2 or 4
  int R = 4;
  std::complex<T> a[16];
};
// A: the products applied to the state (forward and uncompute), in the wide type; D: the
// pull-back products and the gradient reconstruction, in double (their rounding stays within
// the reference's floors in both precisions, tests/floors.py)
using SMat = SMatT<hreal>;
using SMatD = SMatT<double>;
using cd = std::complex<hreal>;
using cdd = std::complex<double>;

template <class T = hreal>
inline SMatT<T> smat_identity(int R) {
  SMatT<T> m;
  m.R = R;
  for (int i = 0; i < R * R; ++i) m.a[i] = 0;
  for (int i = 0; i < R; ++i) m.a[i * R + i] = 1;
  return m;
}
template <class T>
inline SMatT<T> smat_mul(const SMatT<T>& x, const SMatT<T>& y) {
  SMatT<T> z;
  z.R = x.R;
  const int R = x.R;
  for (int p = 0; p < R; ++p)
    for (int q = 0; q < R; ++q) {
      T sr = 0, si = 0;  // (real arithmetic: no complex-multiply NaN/Inf recovery path)
      for (int k = 0; k < R; ++k) {
        const std::complex<T> u = x.a[p * R + k], v = y.a[k * R + q];
        sr += u.real() * v.real() - u.imag() * v.imag();
        si += u.real() * v.imag() + u.imag() * v.real();
      }
      z.a[p * R + q] = std::complex<T>(sr, si);
    }
  return z;
}
template <class T>
inline SMatT<T> smat_transpose(const SMatT<T>& x) {
  SMatT<T> z;
  z.R = x.R;
  for (int p = 0; p < x.R; ++p)
    for (int q = 0; q < x.R; ++q) z.a[p * x.R + q] = x.a[q * x.R + p];
  return z;
}
// the same matrix in double
template <class T>
inline SMatD smat_double(const SMatT<T>& x) {
  SMatD z;
  z.R = x.R;
  for (int i = 0; i < x.R * x.R; ++i) z.a[i] = cdd((double)x.a[i].real(), (double)x.a[i].imag());
  return z;
}

// swap of the two qubit bits of a 4-index: (2h + l) -> (2l + h)
inline int swap_bits4(int r) { return ((r & 1) << 1) | (r >> 1); }

// How one gate sits in its stage.
enum StageRole : int {
  ROLE_Q1_ONLY = 0,  // one-qubit gate in a one-qubit stage
  ROLE_Q1_LO = 1,    // one-qubit gate on the stage's lo qubit
  ROLE_Q1_HI = 2,    // ... on the hi qubit
  ROLE_Q2 = 3,       // two-qubit gate with pos2 = hi, pos1 = lo (stage basis == gate basis)
  ROLE_Q2_SWAP = 4,  // two-qubit gate with pos2 = lo, pos1 = hi
};

// Embed a gate's matrix (its own basis; R_g = 2 or 4 entries row-major, or a diagonal of 4 when
// `diag`) into the stage basis of dimension R.
template <class T>
inline SMatT<T> stage_embed(const std::complex<T>* g, bool diag, int role, int R) {
  SMatT<T> m = smat_identity<T>(R);
  if (role == ROLE_Q1_ONLY) {
    for (int i = 0; i < 4; ++i) m.a[i] = g[i];
    return m;
  }
  for (int i = 0; i < 16; ++i) m.a[i] = 0;
  if (role == ROLE_Q1_LO || role == ROLE_Q1_HI) {
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        const int rh = r >> 1, rl = r & 1, ch = c >> 1, cl = c & 1;
        if (role == ROLE_Q1_LO)
          m.a[r * 4 + c] = (rh == ch) ? g[rl * 2 + cl] : std::complex<T>(0);
        else
          m.a[r * 4 + c] = (rl == cl) ? g[rh * 2 + ch] : std::complex<T>(0);
      }
    return m;
  }
  const bool sw = role == ROLE_Q2_SWAP;
  for (int r = 0; r < 4; ++r) {
    const int gr = sw ? swap_bits4(r) : r;
    if (diag) {
      m.a[r * 4 + r] = g[gr];
    } else {
      for (int c = 0; c < 4; ++c) m.a[r * 4 + c] = g[gr * 4 + (sw ? swap_bits4(c) : c)];
    }
  }
  return m;
}

// Gradient of one gate (its own index order) from M = L Gamma Rt in the stage basis.
// Writes 4 (q1, diagonal) or 16 (two-qubit) complex values.
inline void stage_extract(const SMatD& M, bool diag, int role, cdd* out) {
  if (role == ROLE_Q1_ONLY) {
    for (int i = 0; i < 4; ++i) out[i] = M.a[i];
    return;
  }
  if (role == ROLE_Q1_LO || role == ROLE_Q1_HI) {
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) {
        cdd s = 0;
        for (int k = 0; k < 2; ++k) {
          const int r = role == ROLE_Q1_LO ? 2 * k + i : 2 * i + k;
          const int c = role == ROLE_Q1_LO ? 2 * k + j : 2 * j + k;
          s += M.a[r * 4 + c];
        }
        out[i * 2 + j] = s;
      }
    return;
  }
  const bool sw = role == ROLE_Q2_SWAP;
  if (diag) {
    for (int p = 0; p < 4; ++p) {
      const int r = sw ? swap_bits4(p) : p;
      out[p] = M.a[r * 4 + r];
    }
    return;
  }
  for (int p = 0; p < 4; ++p)
    for (int q = 0; q < 4; ++q) {
      const int r = sw ? swap_bits4(p) : p, c = sw ? swap_bits4(q) : q;
      out[p * 4 + q] = M.a[r * 4 + c];
    }
}

// One variable gate's gradient recipe inside a stage.
struct StageGate {
  uint32_t var;  // row of the gradient output (variable-gate order)
  bool diag;
  int role;
  SMatD L, Rt;  // G_stage = L Gamma Rt
};

// A stage whose Gamma is reduced into gradient slot `slot`.
struct StagePost {
  uint32_t slot;
  int R;           // 2 or 4
  bool diag_only;  // Gamma holds only its diagonal (4 values)
  // register-resident pass run with t1/t2 exchanged (slot case S1 < S2, qdc_rq.hpp): the
  // kernel's Gamma index bits are swapped (Gamma[p][q] = got[swap p][swap q])
  bool swapped = false;
  std::vector<StageGate> gates;
};

}  // namespace qdc
