"""LANE-family single-gate kernels (k_lane: one chunk per lane, partner amplitudes across
lanes; csrc/qdc_kernels.hpp) against the oracle at every target placement of small states:
each q1 position and every ordered q2 pair at n = 7 (one 64-chunk unit in f32), 9, 12 and 14
(the block-wide variant's 1024-chunk units from n = 11 in f32) — targets inside the chunk (f32
qubit 0), at near lane bits and at far lane bits — for gate
application, densities and gradients (primitives.cu:513-646, 689-837, 202-354 via the
primitives ABI).  Tolerances as test_gpu_primitives: 1e-5 (f32), 1e-12 (f64) relative."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

TOL = {"f32": 1e-5, "f64": 1e-12}
DT = {"f32": np.complex64, "f64": np.complex128}


def rnd(rng, size, prec):
    return (rng.random(size) + 1j * rng.random(size)).astype(DT[prec])


def relerr(got, want):
    got = np.asarray(got, dtype=np.complex128).reshape(-1)
    want = np.asarray(want, dtype=np.complex128).reshape(-1)
    return float(np.abs(got - want).max() / max(np.abs(want).max(), 1e-300))


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [7, 9, 12, 14])
def test_lane_kernels_every_placement(prec, n):
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(100 + n)
    st = rnd(rng, 1 << n, prec)
    bw = rnd(rng, 1 << n, prec)
    s64, b64 = st.astype(np.complex128), bw.astype(np.complex128)
    fwd = q.QuantizedTensor.new_from_host(st, prec)
    bwd = q.QuantizedTensor.new_from_host(bw, prec)
    bad = []
    for pos in range(n):
        g = rnd(rng, 4, prec)
        vm = q.QuantizedTensor.new_from_host(st, prec)
        vm.apply_q1_gate(g, pos)
        checks = {
            "apply": (vm.get_cpu_state_copy(), O.apply_q1_gate(s64, g.astype(np.complex128), pos)),
            "density": (fwd.get_q1_density(pos), O.get_q1_density(s64, pos)),
            "grad": (q.get_q1_grad(fwd, bwd, pos), O.get_q1_grad(s64, b64, pos)),
        }
        for k, (got, want) in checks.items():
            e = relerr(got, want)
            if not e <= TOL[prec]:
                bad.append(f"q1 {k} pos={pos} err={e:.2e}")
    for pos2 in range(n):
        for pos1 in range(n):
            if pos2 == pos1:
                continue
            g = rnd(rng, 16, prec)
            vm = q.QuantizedTensor.new_from_host(st, prec)
            vm.apply_q2_gate(g, pos2, pos1)
            checks = {
                "apply": (vm.get_cpu_state_copy(),
                          O.apply_q2_gate(s64, g.astype(np.complex128), pos2, pos1)),
                "density": (fwd.get_q2_density(pos2, pos1), O.get_q2_density(s64, pos2, pos1)),
                "grad": (q.get_q2_grad(fwd, bwd, pos2, pos1), O.get_q2_grad(s64, b64, pos2, pos1)),
            }
            for k, (got, want) in checks.items():
                e = relerr(got, want)
                if not e <= TOL[prec]:
                    bad.append(f"q2 {k} ({pos2},{pos1}) err={e:.2e}")
    assert not bad, f"{len(bad)} failing cells: " + "; ".join(bad[:40])
