"""The reference's own host call sequence over the 18-function C ABI.

``AbiCircuit`` restates ``src/circuit.rs:164-429`` (``run``, ``forward``, ``backward``) step by
step over ``QuantizedTensor`` (``src/quantized_tensor.rs:54-238``), i.e. over exactly the C ABI a
Rust host linking ``libqdc_{f32,f64}.so`` in place of the CUDA ``libprimitives.a`` calls
(``src/primitives_bind.rs:15-119``):

* forward: one ``q1gate`` / ``q2gate`` / ``q2gate_diag`` per gate, ``get_q*density`` (a host
  sync each) per density;
* backward, per gate: ``apply_*_conj_tr`` (or ``*_inv``) on fwd, then for a variable gate
  ``get_q*_grad`` (a reduction + host sync), then ``apply_*_tr`` on bwd; per density cotangent:
  ``conj_and_double`` into a freshly allocated state, ``apply_*_tr`` on it, ``add`` into bwd,
  and the temporary is dropped.

No fusion, no device-resident gradients: this is the path the circuit runtime
(``qdc_circuit_*``, ``Circuit``) replaces, kept to prove the primitive ABI drop-in end to end
(tests/test_gpu_abi_replay.py) and to time it (bench.py ``abi_unfused``).  Panics follow
circuit.rs; the instruction kinds are those of ``include/qdc/circuit.h``.
"""
from __future__ import annotations

from collections import deque
from typing import List

import numpy as np

from . import (CONST_Q1, CONST_Q1_NONU, CONST_Q2, CONST_Q2_DIAG, CONST_Q2_NONU,
               DIFF_Q1_DENSITY, DIFF_Q2_DENSITY, PanicException, Q1_DENSITY, Q2_DENSITY,
               QuantizedTensor, VAR_Q1, VAR_Q1_NONU, VAR_Q2, VAR_Q2_DIAG, VAR_Q2_NONU,
               data_transfer, get_q1_grad, get_q2_grad, get_q2_grad_diag)

_CONST = (CONST_Q1, CONST_Q1_NONU, CONST_Q2, CONST_Q2_NONU, CONST_Q2_DIAG)
_VAR = (VAR_Q1, VAR_Q1_NONU, VAR_Q2, VAR_Q2_NONU, VAR_Q2_DIAG)
_Q1 = (CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU)
_Q2 = (CONST_Q2, CONST_Q2_NONU, VAR_Q2, VAR_Q2_NONU)
_NONU = (CONST_Q1_NONU, CONST_Q2_NONU, VAR_Q1_NONU, VAR_Q2_NONU)


def _slice(a, msg="Gate is not contiguous."):
    """PyReadonlyArray::as_slice().expect(msg)."""
    a = np.asarray(a)
    if not a.flags.c_contiguous:
        raise PanicException(msg)
    return a.reshape(-1)


class AbiCircuit:
    """circuit.rs's ``Circuit`` (new, set_state_from_vector, add_*, run, forward, backward)."""

    def __init__(self, qubits_number: int, precision: str | None = None):
        # Circuit::new (circuit.rs:95-103): |0..0> and a clone of it
        self.initial_state = QuantizedTensor.new_standard(qubits_number, precision)
        self.state = self.initial_state.clone()
        self.instructions = []
        self.dtype = self.initial_state.dtype

    def set_state_from_vector(self, vector):
        self.initial_state.set_from_host(np.asarray(vector, dtype=self.dtype))

    def add(self, kind, *pos):
        self.instructions.append((int(kind), tuple(int(p) for p in pos)))

    # --- circuit.rs:164-264 -------------------------------------------------------------
    def _forward(self, const_gates, var_gates, all_densities) -> List[np.ndarray]:
        if not self.instructions:
            raise PanicException("The circuit is empty.")
        out = []
        cg, vg = deque(const_gates), deque(var_gates)
        data_transfer(self.initial_state, self.state)
        s = self.state
        for kind, pos in self.instructions:
            if kind in _CONST or kind in _VAR:
                pool = cg if kind in _CONST else vg
                if not pool:
                    word = "constant" if kind in _CONST or kind == VAR_Q2_DIAG else "variable"
                    raise PanicException(f"The number of {word} gates is less than required.")
                g = _slice(pool.popleft())
                if kind in _Q1:
                    s.apply_q1_gate(g, pos[0])
                elif kind in _Q2:
                    s.apply_q2_gate(g, *pos)
                else:
                    s.apply_q2_gate_diag(g, *pos)
            elif kind in (DIFF_Q1_DENSITY, DIFF_Q2_DENSITY) or (
                    all_densities and kind in (Q1_DENSITY, Q2_DENSITY)):
                if kind in (Q1_DENSITY, DIFF_Q1_DENSITY):
                    out.append(s.get_q1_density(pos[0]).reshape(2, 2))
                else:
                    out.append(s.get_q2_density(*pos).reshape(4, 4))
        if cg:
            raise PanicException("Number of constant gates is more than required.")
        if vg:
            raise PanicException("Number of variable gates is more than required.")
        return out

    def run(self, const_gates, var_gates):
        return self._forward(const_gates, var_gates, True)

    def forward(self, const_gates, var_gates):
        return self._forward(const_gates, var_gates, False)

    # --- circuit.rs:266-429 -------------------------------------------------------------
    def backward(self, grads_wrt_density, const_gates, var_gates) -> List[np.ndarray]:
        if not self.instructions:
            raise PanicException("The circuit is empty.")
        dens, cg, vg = list(grads_wrt_density), list(const_gates), list(var_gates)
        fwd = self.state
        bwd = None
        grads = deque()
        for kind, pos in reversed(self.instructions):
            if kind in _CONST or kind in _VAR:
                pool = cg if kind in _CONST else vg
                if not pool:
                    raise PanicException("The number of gates is less than required.")
                g = _slice(pool.pop())
                if kind in _Q1:
                    (fwd.apply_q1_gate_inv if kind in _NONU else fwd.apply_q1_gate_conj_tr)(g, pos[0])
                elif kind in _Q2:
                    (fwd.apply_q2_gate_inv if kind in _NONU else fwd.apply_q2_gate_conj_tr)(g, *pos)
                else:
                    fwd.apply_q2_gate_diag_conj(g, *pos)
                if bwd is not None:
                    if kind in _VAR:
                        if kind in _Q1:
                            grads.appendleft(get_q1_grad(fwd, bwd, pos[0]))
                        elif kind in _Q2:
                            grads.appendleft(get_q2_grad(fwd, bwd, *pos))
                        else:
                            grads.appendleft(get_q2_grad_diag(fwd, bwd, *pos))
                    if kind in _Q1:
                        bwd.apply_q1_gate_tr(g, pos[0])
                    elif kind in _Q2:
                        bwd.apply_q2_gate_tr(g, *pos)
                    else:
                        bwd.apply_q2_gate_diag(g, *pos)
                elif kind in _VAR:
                    grads.appendleft(np.zeros(16 if kind in _Q2 else 4, self.dtype))
            elif kind in (DIFF_Q1_DENSITY, DIFF_Q2_DENSITY):
                if not dens:
                    raise PanicException(
                        "The number of gradients wrt density matrices is less than required.")
                gd = _slice(dens.pop(), "Gradient is not contiguous.")
                addition = fwd.conj_and_double()  # a new state (quantized_tensor.rs:81-86)
                if kind == DIFF_Q1_DENSITY:
                    addition.apply_q1_gate_tr(gd, pos[0])
                else:
                    addition.apply_q2_gate_tr(gd, *pos)
                if bwd is None:
                    bwd = addition
                else:
                    bwd.add(addition)  # consumes and drops `addition` (quantized_tensor.rs:87-90)
                    del addition
        if cg:
            raise PanicException("Number of constant gates is more than required.")
        if vg:  # circuit.rs:426
            raise PanicException("Number of constant gates is more than required.")
        if dens:
            raise PanicException("Number of gradients wrt density matrices is more than required.")
        self.bwd = bwd
        return list(grads)
