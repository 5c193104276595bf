"""CPU oracle for the differentiable state-vector hot path — TEST INFRASTRUCTURE ONLY.

This module restates, in numpy, what the reference computes on its hot path:

* the primitive ops, written exactly like the reference's own einsum test oracles
  (``src/quantized_tensor.rs:287-398``) — which SURVEY.md §0/§8c verified to equal the CUDA
  kernel index rules of ``src/primitives.cu:202-953``;
* the inverse used by the ``*NonU`` uncompute (``src/primitives.cu:114-138``);
* the ``Circuit`` interpreter — ``run`` / ``forward`` / the O(1)-memory ``backward`` — of
  ``src/circuit.rs:164-429`` including its panic messages, FIFO/LIFO gate consumption and the
  zero gradients of variable gates met before any density cotangent;
* the reference's comparison metric ``cmp_complex_slices`` (``src/test_utils.rs:20-42``).

Pinning: the reference ships no golden vectors and cannot be built or imported here
(CUDA + Rust/PyO3 + JAX).  This oracle is pinned by the reference's own
known-answer tests — the GHZ amplitudes and densities of ``primitives.cu:979-1029``,
``quantized_tensor.rs:487-506`` and ``test_ghz.py:32-60``, the inverse KAT of
``primitives.cu:1035-1073`` — and by the finite-difference gradient identity of
``test_autodiff.py:152-165`` (see ``tests/test_oracle.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this package; the product path (``differentiable-quantum-circuit-cuda_amd``) never does.
"""
from __future__ import annotations

import numpy as np

# Instruction kinds, in the order of `enum Instruction` (src/circuit.rs:53-68)
CONST_Q2, VAR_Q2, CONST_Q2_NONU, VAR_Q2_NONU, CONST_Q2_DIAG, VAR_Q2_DIAG = range(6)
CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU = range(6, 10)
Q2_DENSITY, Q1_DENSITY, DIFF_Q2_DENSITY, DIFF_Q1_DENSITY = range(10, 14)


class OraclePanic(Exception):
    """Mirrors a Rust `panic!` / `assert!` of the reference (surfaced by PyO3)."""


def qubits_of(size: int) -> int:
    """get_qubits_number (quantized_tensor.rs:44-52)."""
    if size == 0 or size & (size - 1):
        raise OraclePanic("State size is not a power of 2.")
    return size.bit_length() - 1


# ---------------------------------------------------------------------------------------
# Primitives (quantized_tensor.rs:287-398)
# ---------------------------------------------------------------------------------------
def apply_q1_gate(state, gate, pos):
    """quantized_tensor.rs:287-294: einsum("iqk,jq->ijk")."""
    n = qubits_of(state.size)
    s = state.reshape(1 << (n - pos - 1), 2, 1 << pos)
    g = np.asarray(gate).reshape(2, 2)
    return np.einsum("iqk,jq->ijk", s, g).reshape(-1)


def _split5(state, pos2, pos1):
    n = qubits_of(state.size)
    mx, mn = max(pos2, pos1), min(pos2, pos1)
    return state.reshape(1 << (n - mx - 1), 2, 1 << (mx - mn - 1), 2, 1 << mn)


def apply_q2_gate(state, gate, pos2, pos1):
    """quantized_tensor.rs:296-308 (pos2 is the MSB of the gate's local index)."""
    s = _split5(state, pos2, pos1)
    g = np.asarray(gate).reshape(2, 2, 2, 2)
    if pos2 > pos1:
        return np.einsum("iqkpm,jlqp->ijklm", s, g).reshape(-1)
    return np.einsum("iqkpm,ljpq->ijklm", s, g).reshape(-1)


def apply_q2_gate_diag(state, gate, pos2, pos1):
    """quantized_tensor.rs:310-322."""
    s = _split5(state, pos2, pos1)
    g = np.asarray(gate).reshape(2, 2)
    if pos2 > pos1:
        return np.einsum("ijklm,jl->ijklm", s, g).reshape(-1)
    return np.einsum("ijklm,lj->ijklm", s, g).reshape(-1)


def apply_qk_gate(state, gate, positions):
    """Dense k-qubit gate (include/qdc/dense.h; no reference counterpart — the convention
    extends apply_q2_gate's: local index bit (k-1-b) is qubit positions[b], positions[0] the
    most significant).  Parity unpinned beyond k = 2, where it must equal apply_q2_gate
    (tests/test_oracle.py checks that)."""
    n = qubits_of(state.size)
    k = len(positions)
    psi = np.asarray(state).reshape([2] * n)  # axis a = qubit n-1-a
    u = np.asarray(gate).reshape([2] * (2 * k))  # out bits then in bits, MSB first
    axes = [n - 1 - p for p in positions]
    out = np.tensordot(u, psi, axes=(list(range(k, 2 * k)), axes))
    # out axes: the k gate outputs (positions order), then psi's other axes in order
    rest = [a for a in range(n) if a not in axes]
    return np.transpose(out, np.argsort(axes + rest)).reshape(-1)


def get_q1_density(state, pos):
    """quantized_tensor.rs:324-332: rho[2q+p] = sum psi[q] conj(psi[p])."""
    n = qubits_of(state.size)
    s = state.reshape(1 << (n - pos - 1), 2, 1 << pos)
    return np.einsum("iqj,ipj->qp", s, s.conj()).reshape(-1)


def get_q2_density(state, pos2, pos1):
    """quantized_tensor.rs:334-347."""
    s = _split5(state, pos2, pos1)
    if pos2 > pos1:
        return np.einsum("iqkpm,irksm->qprs", s, s.conj()).reshape(-1)
    return np.einsum("iqkpm,irksm->pqsr", s, s.conj()).reshape(-1)


def get_q1_grad(fwd, bwd, pos):
    """quantized_tensor.rs:349-357: G[2q+p] = sum bwd[q] fwd[p]."""
    n = qubits_of(fwd.size)
    f = fwd.reshape(1 << (n - pos - 1), 2, 1 << pos)
    b = bwd.reshape(1 << (n - pos - 1), 2, 1 << pos)
    return np.einsum("iqj,ipj->qp", b, f).reshape(-1)


def get_q2_grad(fwd, bwd, pos2, pos1):
    """quantized_tensor.rs:359-372."""
    f, b = _split5(fwd, pos2, pos1), _split5(bwd, pos2, pos1)
    if pos2 > pos1:
        return np.einsum("iqkpm,irksm->qprs", b, f).reshape(-1)
    return np.einsum("iqkpm,irksm->pqsr", b, f).reshape(-1)


def get_q2_grad_diag(fwd, bwd, pos2, pos1):
    """quantized_tensor.rs:374-387."""
    f, b = _split5(fwd, pos2, pos1), _split5(bwd, pos2, pos1)
    if pos2 > pos1:
        return np.einsum("iqkpm,iqkpm->qp", b, f).reshape(-1)
    return np.einsum("iqkpm,iqkpm->pq", b, f).reshape(-1)


def conj_and_double(state):
    """quantized_tensor.rs:389-391."""
    return 2 * state.conj()


def add(src, dst):
    """quantized_tensor.rs:393-398: dst += src."""
    return dst + src


def inverse(gate):
    """cublas{C,Z}matinvBatched as called by primitives.cu:114-138 (LU with partial pivoting of
    the column-major view; a zero pivot raises "U(i, i) is zero.")."""
    k = int(round(np.sqrt(np.asarray(gate).size)))
    a = np.asarray(gate, dtype=np.complex128).reshape(k, k)
    m = a.T.copy()  # the column-major view cuBLAS factorises
    for j in range(k):
        piv = j + int(np.argmax(np.abs(m[j:, j])))
        if m[piv, j] == 0:
            raise OraclePanic(f"U({j + 1}, {j + 1}) is zero.")
        if piv != j:
            m[[j, piv]] = m[[piv, j]]
        m[j + 1:, j:] -= np.outer(m[j + 1:, j] / m[j, j], m[j, j:])
    return np.linalg.inv(a).reshape(-1)


def transpose(gate):
    """apply_q*_gate_tr (quantized_tensor.rs:110-114, 134-139)."""
    k = int(round(np.sqrt(np.asarray(gate).size)))
    return np.asarray(gate).reshape(k, k).T.reshape(-1)


def conj_transpose(gate):
    """apply_q*_gate_conj_tr (quantized_tensor.rs:115-119, 140-145)."""
    return transpose(gate).conj()


def cmp_complex_slices(lhs, rhs, tol):
    """test_utils.rs:20-42: per element |a-b| / max(|a|,|b|) < tol, pairs of zeros skipped.
    Returns the worst relative error; raises AssertionError like the reference's panic."""
    lhs = np.asarray(lhs).reshape(-1)
    rhs = np.asarray(rhs).reshape(-1)
    assert lhs.shape == rhs.shape, (lhs.shape, rhs.shape)
    mx = np.maximum(np.abs(lhs), np.abs(rhs))
    nz = mx != 0
    rel = np.zeros(lhs.shape, dtype=np.float64)
    rel[nz] = np.abs(lhs[nz] - rhs[nz]) / mx[nz]
    worst = float(rel.max()) if rel.size else 0.0
    if not worst < tol:
        idx = int(rel.argmax())
        raise AssertionError(
            f"Elements number {idx} are too different: lhs: {lhs[idx]}, rhs: {rhs[idx]} "
            f"(rel {worst:.3e} >= {tol:.1e})")
    return worst


# ---------------------------------------------------------------------------------------
# Circuit interpreter (circuit.rs:86-429)
# ---------------------------------------------------------------------------------------
_Q1_GATES = (CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU)
_Q2_DENSE = (CONST_Q2, VAR_Q2, CONST_Q2_NONU, VAR_Q2_NONU)
_DIAG = (CONST_Q2_DIAG, VAR_Q2_DIAG)
_CONST = (CONST_Q1, CONST_Q1_NONU, CONST_Q2, CONST_Q2_NONU, CONST_Q2_DIAG)
_VAR = (VAR_Q1, VAR_Q1_NONU, VAR_Q2, VAR_Q2_NONU, VAR_Q2_DIAG)
_NONU = (CONST_Q1_NONU, VAR_Q1_NONU, CONST_Q2_NONU, VAR_Q2_NONU)


def _check_gate(kind, pos, gate, n):
    """The asserts of QuantizedTensor::apply_* (quantized_tensor.rs:100-152)."""
    want = 16 if kind in _Q2_DENSE else 4
    if gate.size != want:
        raise OraclePanic("Incorrect len of the gate's buffer.")
    if kind in _Q1_GATES:
        if pos[0] >= n:
            raise OraclePanic("pos is out of the bound.")
    else:
        pos2, pos1 = pos
        if pos1 == pos2:
            raise OraclePanic("pos1 and pos2 must be different.")
        if pos1 >= n:
            raise OraclePanic("pos1 is out of the bound.")
        if pos2 >= n:
            raise OraclePanic("pos2 is out of the bound.")


class EinsumOps:
    """The einsum restatements above, as an op table (state held in complex128)."""
    state_dtype = np.dtype(np.complex128)
    apply_q1_gate = staticmethod(apply_q1_gate)
    apply_q2_gate = staticmethod(apply_q2_gate)
    apply_q2_gate_diag = staticmethod(apply_q2_gate_diag)
    get_q1_density = staticmethod(get_q1_density)
    get_q2_density = staticmethod(get_q2_density)
    get_q1_grad = staticmethod(get_q1_grad)
    get_q2_grad = staticmethod(get_q2_grad)
    get_q2_grad_diag = staticmethod(get_q2_grad_diag)
    conj_and_double = staticmethod(conj_and_double)
    add = staticmethod(add)


class OracleCircuit:
    """A restatement of the reference's `Circuit` pyclass (circuit.rs:86-430) over an op table:
    `EinsumOps` (numpy, complex128 state) or `oracle.cref.CRefOps` (the C/OpenMP restatement of
    the CUDA kernels, in the build's precision).  `dtype` fixes the dtype of returned arrays.
    """

    def __init__(self, qubits_number: int, dtype=np.complex128, ops=EinsumOps):
        self.n = qubits_number
        self.dtype = np.dtype(dtype)
        self.ops = ops
        self.instructions = []
        self.initial_state = np.zeros(1 << qubits_number, dtype=ops.state_dtype)
        self.initial_state[0] = 1
        self.state = self.initial_state.copy()
        self.bwd = None

    # builders (circuit.rs:104-162)
    def set_state_from_vector(self, vector):
        v = np.asarray(vector)
        if qubits_of(v.size) != self.n:
            raise OraclePanic("Size of the given state does not match the size of the tensor.")
        self.initial_state = v.astype(self.ops.state_dtype).reshape(-1)

    def add(self, kind, *pos):
        self.instructions.append((kind, tuple(pos)))

    def add_q2_const_gate(self, pos2, pos1): self.add(CONST_Q2, pos2, pos1)
    def add_q2_const_gate_diag(self, pos2, pos1): self.add(CONST_Q2_DIAG, pos2, pos1)
    def add_q2_const_gate_nonu(self, pos2, pos1): self.add(CONST_Q2_NONU, pos2, pos1)
    def add_q2_var_gate(self, pos2, pos1): self.add(VAR_Q2, pos2, pos1)
    def add_q2_var_gate_diag(self, pos2, pos1): self.add(VAR_Q2_DIAG, pos2, pos1)
    def add_q2_var_gate_nonu(self, pos2, pos1): self.add(VAR_Q2_NONU, pos2, pos1)
    def add_q1_const_gate(self, pos): self.add(CONST_Q1, pos)
    def add_q1_const_gate_nonu(self, pos): self.add(CONST_Q1_NONU, pos)
    def add_q1_var_gate(self, pos): self.add(VAR_Q1, pos)
    def add_q1_var_gate_nonu(self, pos): self.add(VAR_Q1_NONU, pos)
    def get_q2_dens_op(self, pos2, pos1): self.add(Q2_DENSITY, pos2, pos1)
    def get_q1_dens_op(self, pos): self.add(Q1_DENSITY, pos)
    def get_q2_dens_op_with_grad(self, pos2, pos1): self.add(DIFF_Q2_DENSITY, pos2, pos1)
    def get_q1_dens_op_with_grad(self, pos): self.add(DIFF_Q1_DENSITY, pos)

    def _apply(self, state, kind, pos, gate):
        _check_gate(kind, pos, gate, self.n)
        gate = np.asarray(gate, dtype=self.ops.state_dtype)
        if kind in _Q1_GATES:
            return self.ops.apply_q1_gate(state, gate, pos[0])
        if kind in _Q2_DENSE:
            return self.ops.apply_q2_gate(state, gate, *pos)
        return self.ops.apply_q2_gate_diag(state, gate, *pos)

    def _density(self, kind, pos):
        if kind in (Q1_DENSITY, DIFF_Q1_DENSITY):
            return self.ops.get_q1_density(self.state, pos[0]).reshape(2, 2)
        return self.ops.get_q2_density(self.state, *pos).reshape(4, 4)

    def _forward(self, const_gates, var_gates, all_densities):
        """circuit.rs:164-264."""
        if not self.instructions:
            raise OraclePanic("The circuit is empty.")
        const_gates = [np.asarray(g).reshape(-1) for g in const_gates]
        var_gates = [np.asarray(g).reshape(-1) for g in var_gates]
        ci = vi = 0
        out = []
        self.state = self.initial_state.copy()
        for kind, pos in self.instructions:
            if kind in _CONST:
                if ci >= len(const_gates):
                    raise OraclePanic("The number of constant gates is less than required.")
                self.state = self._apply(self.state, kind, pos, const_gates[ci])
                ci += 1
            elif kind in _VAR:
                if vi >= len(var_gates):
                    # circuit.rs:198 / :249 say "constant" for VarQ2GateDiag
                    word = "constant" if kind == VAR_Q2_DIAG else "variable"
                    raise OraclePanic(f"The number of {word} gates is less than required.")
                self.state = self._apply(self.state, kind, pos, var_gates[vi])
                vi += 1
            elif kind in (DIFF_Q1_DENSITY, DIFF_Q2_DENSITY) or all_densities:
                out.append(self._density(kind, pos).astype(self.dtype))
        if ci != len(const_gates):
            raise OraclePanic("Number of constant gates is more than required.")
        if vi != len(var_gates):
            raise OraclePanic("Number of variable gates is more than required.")
        return out

    def run(self, const_gates, var_gates):
        return self._forward(const_gates, var_gates, True)

    def forward(self, const_gates, var_gates):
        return self._forward(const_gates, var_gates, False)

    def backward(self, grads_wrt_density, const_gates, var_gates):
        """circuit.rs:266-429: reverse sweep from the final forward state."""
        if not self.instructions:
            raise OraclePanic("The circuit is empty.")
        dens = [np.asarray(g).reshape(-1) for g in grads_wrt_density]
        const_gates = [np.asarray(g).reshape(-1) for g in const_gates]
        var_gates = [np.asarray(g).reshape(-1) for g in var_gates]
        fwd = self.state
        bwd = None
        grads = []
        for kind, pos in reversed(self.instructions):
            if kind in _CONST or kind in _VAR:
                pool = const_gates if kind in _CONST else var_gates
                if not pool:
                    raise OraclePanic("The number of gates is less than required.")
                g = pool.pop()
                if kind in _DIAG:
                    fwd = self._apply(fwd, kind, pos, g.conj())
                elif kind in _NONU:
                    _check_gate(kind, pos, g, self.n)
                    fwd = self._apply(fwd, kind, pos, inverse(g))
                else:
                    fwd = self._apply(fwd, kind, pos, conj_transpose(g))
                if bwd is not None:
                    if kind in _VAR:
                        if kind in _Q1_GATES:
                            grads.insert(0, self.ops.get_q1_grad(fwd, bwd, pos[0]))
                        elif kind in _Q2_DENSE:
                            grads.insert(0, self.ops.get_q2_grad(fwd, bwd, *pos))
                        else:
                            grads.insert(0, self.ops.get_q2_grad_diag(fwd, bwd, *pos))
                    bwd = self._apply(bwd, kind, pos, g if kind in _DIAG else transpose(g))
                elif kind in _VAR:
                    grads.insert(0, np.zeros(16 if kind in _Q2_DENSE else 4, self.ops.state_dtype))
            elif kind in (DIFF_Q1_DENSITY, DIFF_Q2_DENSITY):
                if not dens:
                    raise OraclePanic(
                        "The number of gradients wrt density matrices is less than required.")
                gd = dens.pop()
                add_ = self.ops.conj_and_double(fwd)
                if gd.size != (4 if kind == DIFF_Q1_DENSITY else 16):
                    raise OraclePanic("Incorrect len of the gate's buffer.")
                gt = np.asarray(transpose(gd), dtype=self.ops.state_dtype)
                if kind == DIFF_Q1_DENSITY:
                    add_ = self.ops.apply_q1_gate(add_, gt, pos[0])
                else:
                    add_ = self.ops.apply_q2_gate(add_, gt, *pos)
                bwd = add_ if bwd is None else self.ops.add(add_, bwd)
        if const_gates:
            raise OraclePanic("Number of constant gates is more than required.")
        if var_gates:  # circuit.rs:426
            raise OraclePanic("Number of constant gates is more than required.")
        if dens:
            raise OraclePanic("Number of gradients wrt density matrices is more than required.")
        self.state = fwd
        self.bwd = bwd
        return [g.astype(self.dtype) for g in grads]


# ---------------------------------------------------------------------------------------
# Workload generators shared by tests, smoke() and bench.py (SURVEY.md §8 d)
# ---------------------------------------------------------------------------------------
# Workload generators live with the product (bench.py uses them for the GPU workload); the
# oracle re-exports them for the tests.
from quantum_differentiable_circuit.workloads import (  # noqa: E402
    haar_unitary, layered_circuit, random_circuit, random_state)


def autodiff_circuit(n, layers, seed):
    """The test_autodiff.py:49-81 circuit structure (every gate kind), with numpy-seeded gates in
    place of the JAX PRNG (test_autodiff.py:83-120).  Returns (ins, const_gates, var_gates,
    perturbations)."""
    rng = np.random.default_rng(seed)
    cnot = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0], np.complex128)

    def rc(k):
        return rng.standard_normal(k * k) + 1j * rng.standard_normal(k * k)

    def rdu():
        return np.exp(1j * rng.standard_normal(4))

    def rdc():
        return rng.standard_normal(4) + 1j * rng.standard_normal(4)

    ins = []
    for _ in range(layers):
        ins += [(DIFF_Q1_DENSITY, (i,)) for i in range(n)]
        ins += [(DIFF_Q2_DENSITY, (i + 1, i)) for i in range(0, n - 1, 2)]
        ins += [(VAR_Q1, (i,)) for i in range(n)]
        ins += [(VAR_Q2, (i + 1, i)) for i in range(0, n - 1, 2)]
        ins += [(VAR_Q2_DIAG, (i + 1, i)) for i in range(0, n - 1, 2)]
        ins += [(CONST_Q1, (i,)) for i in range(n)]
        ins += [(CONST_Q2, (i + 1, i)) for i in range(1, n - 1, 2)]
        ins += [(CONST_Q2_DIAG, (i + 1, i)) for i in range(1, n - 1, 2)]
        ins += [(VAR_Q1_NONU, (i,)) for i in range(n)]
        ins += [(VAR_Q2_NONU, (i + 1, i)) for i in range(0, n - 1, 2)]
        ins += [(CONST_Q1_NONU, (i,)) for i in range(n)]
        ins += [(CONST_Q2_NONU, (i + 1, i)) for i in range(1, n - 1, 2)]
    ins += [(Q1_DENSITY, (i,)) for i in range(n)]
    ins += [(Q2_DENSITY, (i + 1, i)) for i in range(0, n - 1, 2)]

    half = len(range(0, n - 1, 2))  # == int((n - 1) / 2) of test_autodiff.py for odd n
    nodd = len(range(1, n - 1, 2))
    const, var, pert = [], [], []
    for _ in range(layers):
        const += [haar_unitary(rng, 2) for _ in range(n)]
        const += [cnot.copy() for _ in range(nodd)]
        const += [rdu() for _ in range(nodd)]
        const += [0.01 * rc(2) + haar_unitary(rng, 2) for _ in range(n)]
        const += [0.01 * rc(4) + haar_unitary(rng, 4) for _ in range(nodd)]
    for _ in range(layers):
        var += [haar_unitary(rng, 2) for _ in range(n)]
        var += [haar_unitary(rng, 4) for _ in range(half)]
        var += [rdu() for _ in range(half)]
        var += [0.01 * rc(2) + haar_unitary(rng, 2) for _ in range(n)]
        var += [0.01 * rc(4) + haar_unitary(rng, 4) for _ in range(half)]
    for _ in range(layers):
        pert += [rc(2) for _ in range(n)]
        pert += [rc(4) for _ in range(half)]
        pert += [rdc() for _ in range(half)]
        pert += [rc(2) for _ in range(n)]
        pert += [rc(4) for _ in range(half)]
    return ins, const, var, pert


def tsallis_loss_and_cotangents(densities):
    """av_tsallis of test_autodiff.py:87-92: mean over densities of 1 - tr(rho^2).
    Returns (loss, JAX cotangents d loss / d rho) — the holomorphic derivative -2 rho^T / N,
    which JAX hands to bwd_run (circuit.py:190-197)."""
    m = len(densities)
    loss = sum((1 - np.einsum("ij,ji->", d, d)).real for d in densities) / m
    cots = [-2.0 * d.T / m for d in densities]
    return float(loss), cots
