#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the oracle.

The reference ships no golden vectors and cannot run here (CUDA + Rust/PyO3 + JAX, SURVEY.md
§8c), so the fixtures are produced by the oracle (oracle/oracle.py, numpy einsum restatement
of src/quantized_tensor.rs:287-398 and src/circuit.rs:164-429), whose correctness is pinned
by the reference's known-answer tests in tests/test_oracle.py.  Inputs are seeded; expected
outputs are computed in complex128 from the inputs rounded to the fixture's dtype.

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402

DT = {"f32": np.complex64, "f64": np.complex128}


def flat(gates, dt):
    lens = np.array([g.size for g in gates], dtype=np.int64)
    data = np.concatenate([np.asarray(g, dtype=dt).reshape(-1) for g in gates]) if gates \
        else np.zeros(0, dt)
    return data, lens


def primitives(prec, n=10, seed=101):
    dt = DT[prec]
    rng = np.random.default_rng(seed)
    state = (rng.random(1 << n) + 1j * rng.random(1 << n)).astype(dt)
    bwd = (rng.random(1 << n) + 1j * rng.random(1 << n)).astype(dt)
    s, b = state.astype(np.complex128), bwd.astype(np.complex128)
    out = {"n": np.array(n), "state": state, "bwd": bwd}
    q1 = (rng.random((n, 4)) + 1j * rng.random((n, 4))).astype(dt)
    out["q1_gates"] = q1
    out["q1_out"] = np.stack([O.apply_q1_gate(s, q1[p].astype(np.complex128), p) for p in range(n)])
    out["q1_density"] = np.stack([O.get_q1_density(s, p) for p in range(n)])
    out["q1_grad"] = np.stack([O.get_q1_grad(s, b, p) for p in range(n)])
    pairs = np.array([(1, 0), (0, 1), (0, n - 1), (n - 1, 0), (3, 7), (7, 3), (n - 1, n - 2),
                      (2, 1), (5, 6), (6, 2)], dtype=np.int64)
    out["pairs"] = pairs
    q2 = (rng.random((len(pairs), 16)) + 1j * rng.random((len(pairs), 16))).astype(dt)
    d4 = (rng.random((len(pairs), 4)) + 1j * rng.random((len(pairs), 4))).astype(dt)
    out["q2_gates"], out["diag_gates"] = q2, d4
    out["q2_out"] = np.stack([O.apply_q2_gate(s, q2[i].astype(np.complex128), *pr)
                              for i, pr in enumerate(pairs)])
    out["diag_out"] = np.stack([O.apply_q2_gate_diag(s, d4[i].astype(np.complex128), *pr)
                                for i, pr in enumerate(pairs)])
    out["q2_density"] = np.stack([O.get_q2_density(s, *pr) for pr in pairs])
    out["q2_grad"] = np.stack([O.get_q2_grad(s, b, *pr) for pr in pairs])
    out["diag_grad"] = np.stack([O.get_q2_grad_diag(s, b, *pr) for pr in pairs])
    out["q1_inverse"] = np.stack([O.inverse(q1[p].astype(np.complex128)) for p in range(n)])
    return out


def circuit_fixture(prec, ins, const, var, psi0, cotangent_fn):
    dt = DT[prec]
    n = O.qubits_of(psi0.size)
    const = [np.asarray(g, dtype=dt) for g in const]
    var = [np.asarray(g, dtype=dt) for g in var]
    o = O.OracleCircuit(n, dt)
    for kind, pos in ins:
        o.add(kind, *pos)
    o.set_state_from_vector(psi0.astype(dt))
    run = o.run(const, var)
    fwd = o.forward(const, var)
    cots = [np.asarray(c, dtype=dt) for c in cotangent_fn([d.astype(np.complex128) for d in fwd])]
    grads = o.backward(cots, const, var)
    cf, cl = flat(const, dt)
    vf, vl = flat(var, dt)
    rf, rl = flat(run, dt)
    ff, fl = flat(fwd, dt)
    tf, tl = flat(cots, dt)
    gf, gl = flat(grads, dt)
    kinds = np.array([(k, pos[0], pos[1] if len(pos) > 1 else 0) for k, pos in ins], np.int64)
    return {"n": np.array(n), "instructions": kinds, "psi0": psi0.astype(dt),
            "const": cf, "const_lens": cl, "var": vf, "var_lens": vl,
            "run": rf, "run_lens": rl, "forward": ff, "forward_lens": fl,
            "cotangents": tf, "cotangent_lens": tl, "grads": gf, "grad_lens": gl,
            "final_state": o.state.astype(dt), "final_bwd": o.bwd.astype(dt)}


def tsallis_cots(dens):
    # the qdc wiring conjugates the JAX cotangent before Circuit.backward (circuit.py:193)
    return [c.conj() for c in O.tsallis_loss_and_cotangents(dens)[1]]


def sigma_z_cots(dens):
    return [np.diag([1.0, -1.0]).astype(np.complex128) for _ in dens]


def main():
    for prec in ("f32", "f64"):
        np.savez_compressed(HERE / f"primitives_{prec}.npz", **primitives(prec))
        ins, const, var, _ = O.autodiff_circuit(7, 2, seed=42)
        psi0 = O.random_state(np.random.default_rng(5), 7)
        np.savez_compressed(HERE / f"circuit_autodiff_{prec}.npz",
                            **circuit_fixture(prec, ins, const, var, psi0, tsallis_cots))
        ins, var = O.layered_circuit(8, 3, seed=24)
        psi0 = np.zeros(1 << 8, np.complex128)
        psi0[0] = 1
        np.savez_compressed(HERE / f"circuit_layered_{prec}.npz",
                            **circuit_fixture(prec, ins, [], var, psi0, sigma_z_cots))
    for p in sorted(HERE.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main()
