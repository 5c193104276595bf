"""AutoGradCircuit — the reference's JAX wiring (src/qdc/circuit.py:8-202) over the HIP runtime.

Same constructor, builders, docstring semantics and ``build() -> (simple_run, autodiff_run)``
taking ``(var_gates, const_gates)``.  When JAX is importable, ``autodiff_run`` is the same
``jax.custom_vjp`` as circuit.py:177-201 (forward residuals = the gate lists; the backward
conjugates the density cotangents, circuit.py:193, and returns ``(gate_grads, None)``).
Without JAX (this platform ships none), ``autodiff_run`` is a ``VJPFunction``: calling it runs
the forward pass, and ``autodiff_run.vjp(var_gates, const_gates)`` returns
``(densities, pullback)`` where ``pullback(density_cotangents)`` performs exactly the
custom_vjp backward — so a numpy/scipy caller can chain the gradients by hand.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np

from quantum_differentiable_circuit import circuit_class

try:  # pragma: no cover - JAX is not installed on the MI355X image
    import jax.numpy as jnp  # noqa: F401
    from jax import custom_vjp

    have_jax = True
except Exception:  # noqa: BLE001
    custom_vjp = None
    have_jax = False


class VJPFunction:
    """JAX-free stand-in for a ``custom_vjp`` function (circuit.py:177-201)."""

    def __init__(self, fwd, bwd):
        self._fwd = fwd
        self._bwd = bwd

    def __call__(self, var_gates, const_gates):
        out, _ = self._fwd(var_gates, const_gates)
        return out

    def vjp(self, var_gates, const_gates):
        out, res = self._fwd(var_gates, const_gates)
        return out, (lambda cotangents: self._bwd(res, cotangents))


class AutoGradCircuit:

    def __init__(self, qubits_number: int, precision: str | None = None):
        """Quantum circuit with automatic differentiation."""
        self.circuit = circuit_class(precision)(qubits_number)
        self.dtype = self.circuit.dtype

    def _np(self, x):
        return np.ascontiguousarray(np.asarray(x), dtype=self.dtype)

    def set_state_from_vector(self, vec):
        """Set initial state from an array (circuit.py:14-22)."""
        self.circuit.set_state_from_vector(self._np(vec).reshape(-1))

    # builders: circuit.py:24-158 (positions: qubit 0 is the innermost numpy axis)
    def add_q2_const_gate(self, pos2: int, pos1: int): self.circuit.add_q2_const_gate(pos2, pos1)
    def add_q2_const_gate_nonu(self, pos2: int, pos1: int): self.circuit.add_q2_const_gate_nonu(pos2, pos1)
    def add_q2_const_gate_diag(self, pos2: int, pos1: int): self.circuit.add_q2_const_gate_diag(pos2, pos1)
    def add_q2_var_gate(self, pos2: int, pos1: int): self.circuit.add_q2_var_gate(pos2, pos1)
    def add_q2_var_gate_nonu(self, pos2: int, pos1: int): self.circuit.add_q2_var_gate_nonu(pos2, pos1)
    def add_q2_var_gate_diag(self, pos2: int, pos1: int): self.circuit.add_q2_var_gate_diag(pos2, pos1)
    def add_q1_const_gate(self, pos: int): self.circuit.add_q1_const_gate(pos)
    def add_q1_const_gate_nonu(self, pos: int): self.circuit.add_q1_const_gate_nonu(pos)
    def add_q1_var_gate(self, pos: int): self.circuit.add_q1_var_gate(pos)
    def add_q1_var_gate_nonu(self, pos: int): self.circuit.add_q1_var_gate_nonu(pos)
    def get_q2_dens_op(self, pos2: int, pos1: int): self.circuit.get_q2_dens_op(pos2, pos1)
    def get_q1_dens_op(self, pos: int): self.circuit.get_q1_dens_op(pos)
    def get_q2_dens_op_with_grad(self, pos2: int, pos1: int): self.circuit.get_q2_dens_op_with_grad(pos2, pos1)
    def get_q1_dens_op_with_grad(self, pos: int): self.circuit.get_q1_dens_op_with_grad(pos)

    def build(self) -> Tuple[Callable, Callable]:
        """Returns (simple_run, autodiff_run) — circuit.py:160-202."""
        to_np = self._np

        def simple_run(var_gates: Sequence, const_gates: Sequence) -> List[np.ndarray]:
            return self.circuit.run([to_np(x).reshape(-1) for x in const_gates],
                                    [to_np(x).reshape(-1) for x in var_gates])

        def fwd_run(var_gates, const_gates):
            dens = self.circuit.forward([to_np(x).reshape(-1) for x in const_gates],
                                        [to_np(x).reshape(-1) for x in var_gates])
            return dens, (const_gates, var_gates)

        def bwd_run(res, density_grads):
            const_gates, var_gates = res
            grads = self.circuit.backward(
                [np.ascontiguousarray(np.asarray(x).conj(), dtype=self.dtype) for x in density_grads],
                [to_np(x).reshape(-1) for x in const_gates],
                [to_np(x).reshape(-1) for x in var_gates])
            return grads, None

        if have_jax:  # pragma: no cover
            @custom_vjp
            def autodiff_run(var_gates, const_gates):
                return fwd_run(var_gates, const_gates)[0]

            autodiff_run.defvjp(fwd_run, bwd_run)
            return simple_run, autodiff_run
        return simple_run, VJPFunction(fwd_run, bwd_run)
