"""The HIP path against the committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py from the oracle).  Tolerances: 1e-5 (f32) / 1e-12 (f64) in the
reference's per-element metric for single ops (test_utils.rs:20-42), norm-relative for
reductions; multi-gate circuits within 4x the measured floor (tests/floors.py)."""
from pathlib import Path

import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
TOL = {"f32": 1e-5, "f64": 1e-12}
Q2_KINDS = (0, 1, 2, 3, 4, 5, 10, 12)


def split(data, lens):
    return np.split(data, np.cumsum(lens)[:-1]) if len(lens) else []


def normrel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_golden_primitives(prec):
    import quantum_differentiable_circuit as q
    z = np.load(GOLDEN / f"primitives_{prec}.npz")
    n = int(z["n"])
    tol = TOL[prec]
    for p in range(n):
        vm = q.QuantizedTensor.new_from_host(z["state"], prec)
        vm.apply_q1_gate(z["q1_gates"][p], p)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), z["q1_out"][p], tol)
        O.cmp_complex_slices(vm.clone().get_cpu_state_copy(), z["q1_out"][p], tol)
        src = q.QuantizedTensor.new_from_host(z["state"], prec)
        assert normrel(src.get_q1_density(p), z["q1_density"][p]) < tol
        bw = q.QuantizedTensor.new_from_host(z["bwd"], prec)
        assert normrel(q.get_q1_grad(src, bw, p), z["q1_grad"][p]) < tol
    for i, (p2, p1) in enumerate(z["pairs"]):
        p2, p1 = int(p2), int(p1)
        vm = q.QuantizedTensor.new_from_host(z["state"], prec)
        vm.apply_q2_gate(z["q2_gates"][i], p2, p1)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), z["q2_out"][i], tol)
        vm = q.QuantizedTensor.new_from_host(z["state"], prec)
        vm.apply_q2_gate_diag(z["diag_gates"][i], p2, p1)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), z["diag_out"][i], tol)
        src = q.QuantizedTensor.new_from_host(z["state"], prec)
        bw = q.QuantizedTensor.new_from_host(z["bwd"], prec)
        assert normrel(src.get_q2_density(p2, p1), z["q2_density"][i]) < tol
        assert normrel(q.get_q2_grad(src, bw, p2, p1), z["q2_grad"][i]) < tol
        assert normrel(q.get_q2_grad_diag(src, bw, p2, p1), z["diag_grad"][i]) < tol


@pytest.mark.parametrize("name", ["circuit_autodiff", "circuit_layered"])
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_golden_circuits(name, prec):
    """The fixtures hold complex128 results of the fixture-precision inputs; the HIP path must
    be within 4x the floor of the reference's own algorithm on the same inputs (the C
    restatement of its kernels in `prec`, tests/floors.py)."""
    import quantum_differentiable_circuit as q
    z = np.load(GOLDEN / f"{name}_{prec}.npz")
    n = int(z["n"])
    ins = [(int(k), (int(a), int(b)) if int(k) in Q2_KINDS else (int(a),))
           for k, a, b in z["instructions"]]
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    c.set_state_from_vector(z["psi0"])
    const, var = split(z["const"], z["const_lens"]), split(z["var"], z["var_lens"])
    cots = [x.reshape(int(np.sqrt(x.size)), -1) for x in split(z["cotangents"], z["cotangent_lens"])]
    fl = F.Floor(prec, n, ins, const, var, psi0=z["psi0"], cots=lambda d, dt: cots)
    # the fixtures are the exact results (rounded to `prec`) the floor is measured against
    for key, fix in (("run", "run"), ("forward", "forward"), ("grads", "grads"),
                     ("uncomputed", "final_state"), ("bwd", "final_bwd")):
        assert F.normrel(fl.exact[key], z[fix]) < (1.2e-7 if prec == "f32" else 1e-14), key
    what = f"golden {name} {prec} "
    fl.check("run", c.run(const, var), what)
    fl.check("forward", c.forward(const, var), what)
    grads = c.backward(cots, const, var)
    assert [g.size for g in grads] == list(z["grad_lens"])
    fl.check("grads", grads, what)
    fl.check("uncomputed", c.get_state(0), what)
    fl.check("bwd", c.get_state(2), what)
