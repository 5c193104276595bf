"""Synthetic workloads (SURVEY.md §8 d): seeded gate matrices and instruction lists of the
benchmark configurations.  Product-side so that bench.py's GPU workload does not depend on the
test oracle; oracle/oracle.py re-exports these for the tests.

Instruction kinds follow the reference's `enum Instruction` (src/circuit.rs:53-68)."""
import numpy as np

CONST_Q2, VAR_Q2, CONST_Q2_NONU, VAR_Q2_NONU, CONST_Q2_DIAG, VAR_Q2_DIAG = range(6)
CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU = range(6, 10)
Q2_DENSITY, Q1_DENSITY, DIFF_Q2_DENSITY, DIFF_Q1_DENSITY = range(10, 14)


def haar_unitary(rng, k):
    """QR of a complex Gaussian, as test_autodiff.py:27-31 (no phase fix, like jnp.linalg.qr)."""
    a = rng.standard_normal((k, k)) + 1j * rng.standard_normal((k, k))
    q, _ = np.linalg.qr(a)
    return q.reshape(-1)


def random_state(rng, n, normalise=True):
    v = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
    return v / np.linalg.norm(v) if normalise else v


def layered_circuit(n, layers, seed):
    """Config C2 (SURVEY.md §8 d): per layer a Haar q1 var gate on every qubit, q2 Haar var gates
    on (i+1, i) for even i then for odd i; DiffQ1Density on every qubit at the end.
    Returns (instructions, var_gates)."""
    rng = np.random.default_rng(seed)
    ins, var = [], []
    for _ in range(layers):
        for q in range(n):
            ins.append((VAR_Q1, (q,)))
            var.append(haar_unitary(rng, 2))
        for start in (0, 1):
            for i in range(start, n - 1, 2):
                ins.append((VAR_Q2, (i + 1, i)))
                var.append(haar_unitary(rng, 4))
    for q in range(n):
        ins.append((DIFF_Q1_DENSITY, (q,)))
    return ins, var


def random_circuit(n, ngates, seed, density_every=0):
    """A random circuit over every gate kind on arbitrary (non-adjacent, either order) qubit
    pairs — the random-circuit configuration of SURVEY.md §8 d (C5), also used to exercise the
    runtime's multi-gate fusion.  Every `density_every` gates (0: never) a DiffQ1Density or
    DiffQ2Density on random qubits; DiffQ1Density on every qubit at the end.
    Returns (ins, const_gates, var_gates)."""
    rng = np.random.default_rng(seed)
    ins, const, var = [], [], []
    kinds = [CONST_Q2, VAR_Q2, CONST_Q2_NONU, VAR_Q2_NONU, CONST_Q2_DIAG, VAR_Q2_DIAG,
             CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU]
    for i in range(ngates):
        k = kinds[rng.integers(len(kinds))]
        if k in (CONST_Q1, CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU):
            ins.append((k, (int(rng.integers(n)),)))
            g = haar_unitary(rng, 2)
            if k in (CONST_Q1_NONU, VAR_Q1_NONU):
                g = g + 0.05 * (rng.standard_normal(4) + 1j * rng.standard_normal(4))
        else:
            a, b = (int(x) for x in rng.choice(n, 2, replace=False))
            ins.append((k, (a, b)))
            if k in (CONST_Q2_DIAG, VAR_Q2_DIAG):
                g = np.exp(1j * rng.standard_normal(4))
            else:
                g = haar_unitary(rng, 4)
                if k in (CONST_Q2_NONU, VAR_Q2_NONU):
                    g = g + 0.05 * (rng.standard_normal(16) + 1j * rng.standard_normal(16))
        (const if k in (CONST_Q2, CONST_Q2_NONU, CONST_Q2_DIAG, CONST_Q1, CONST_Q1_NONU)
         else var).append(g)
        if density_every and (i + 1) % density_every == 0:
            if rng.integers(2):
                ins.append((DIFF_Q1_DENSITY, (int(rng.integers(n)),)))
            else:
                a, b = (int(x) for x in rng.choice(n, 2, replace=False))
                ins.append((DIFF_Q2_DENSITY, (a, b)))
    ins += [(DIFF_Q1_DENSITY, (q,)) for q in range(n)]
    return ins, const, var
