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



def brickwall_circuit(n, layers, seed):
    """Config C4 (SURVEY.md §8 d): `layers` layers of Haar q2 variable gates on (i, i+1), even i
    then odd i (so gates on the top qubits straddle the shard boundary when sharded), then
    DiffQ1Density on every qubit.  Returns (instructions, var_gates)."""
    rng = np.random.default_rng(seed)
    ins, var = [], []
    for _ in range(layers):
        for start in (0, 1):
            for i in range(start, n - 1, 2):
                ins.append((VAR_Q2, (i, i + 1)))
                var.append(haar_unitary(rng, 4))
    ins += [(DIFF_Q1_DENSITY, (q,)) for q in range(n)]
    return ins, var


def deep_random_circuit(n, ngates, seed):
    """Config C5 (SURVEY.md §8 d): `ngates` gates, 50 % Haar q1, 35 % Haar q2, 15 % diagonal
    exp(i N(0,1)), all variable, positions uniform and distinct; DiffQ1Density on qubits
    {0, n//2, n-2, n-1} at the end (C5 at n = 33: {0, 16, 31, 32}).
    Returns (instructions, var_gates)."""
    rng = np.random.default_rng(seed)
    ins, var = [], []
    for _ in range(ngates):
        u = rng.random()
        if u < 0.5:
            ins.append((VAR_Q1, (int(rng.integers(n)),)))
            var.append(haar_unitary(rng, 2))
        else:
            a, b = (int(x) for x in rng.choice(n, 2, replace=False))
            if u < 0.85:
                ins.append((VAR_Q2, (a, b)))
                var.append(haar_unitary(rng, 4))
            else:
                ins.append((VAR_Q2_DIAG, (a, b)))
                var.append(np.exp(1j * rng.standard_normal(4)))
    ins += [(DIFF_Q1_DENSITY, (q,)) for q in sorted({0, n // 2, n - 2, n - 1})]
    return ins, var

# ---- config C3: VQSE on the critical transverse-field Ising chain (example_vqse_ising.py) ----

def vqse_ising(n, layers):
    """The example's circuit (example_vqse_ising.py:64-80): per layer a variable diagonal ZZ gate
    on (i, i+1) for i < n-1 and on (0, n-1), then a variable X rotation on every qubit; then
    DiffQ2Density on (i, i+1) and (0, n-1).  Returns the instruction list."""
    ins = []
    for _ in range(layers):
        ins += [(VAR_Q2_DIAG, (i, i + 1)) for i in range(n - 1)] + [(VAR_Q2_DIAG, (0, n - 1))]
        ins += [(VAR_Q1, (i,)) for i in range(n)]
    ins += [(DIFF_Q2_DENSITY, (i, i + 1)) for i in range(n - 1)] + [(DIFF_Q2_DENSITY, (0, n - 1))]
    return ins


def tfim_term(field=1.0):
    """The two-qubit Hamiltonian term of example_vqse_ising.py:88-95:
    -Z⊗Z - field/2 (X⊗1 + 1⊗X), row index = 2 bit(pos2) + bit(pos1)."""
    sz = np.diag([1.0, -1.0]).astype(np.complex128)
    sx = np.array([[0, 1], [1, 0]], dtype=np.complex128)
    eye = np.eye(2, dtype=np.complex128)
    return -np.kron(sz, sz) - 0.5 * field * (np.kron(sx, eye) + np.kron(eye, sx))


def vqse_gates(params, n):
    """params2gates (example_vqse_ising.py:42-49): 2 parameters per layer (gamma, beta) ->
    n zz(gamma) diagonals then n x(beta) rotations, in instruction order."""
    gates = []
    for layer in range(len(params) // 2):
        g, b = float(params[2 * layer]), float(params[2 * layer + 1])
        zz = np.array([np.exp(-1j * g), np.exp(1j * g), np.exp(1j * g), np.exp(-1j * g)])
        x = np.array([np.cos(b), -1j * np.sin(b), -1j * np.sin(b), np.cos(b)])
        gates += [zz] * n + [x] * n
    return gates


def vqse_loss_and_grad(fwd_vjp, params, n, h):
    """Energy sum_k Re tr(rho_k h) and its gradient in the real parameters, the chain
    `value_and_grad(loss)` of example_vqse_ising.py:101-107 written out without JAX.
    fwd_vjp(gates) -> (densities, pullback); pullback(density cotangents) -> (gate cotangents,
    None), the custom_vjp backward (qdc.AutoGradCircuit's VJPFunction.vjp).  The density cotangent of Re tr(rho h) is h^T; a
    real parameter's is Re sum_k c_k dz_k/dparam over its gates (JAX's convention)."""
    gates = vqse_gates(params, n)
    dens, pullback = fwd_vjp(gates)
    e = float(sum(np.real(np.einsum("ij,ji", d, h)) for d in dens))
    cots, _ = pullback([np.ascontiguousarray(h.T) for _ in dens])
    grad = np.zeros(len(params))
    k = 0
    for layer in range(len(params) // 2):
        g, b = float(params[2 * layer]), float(params[2 * layer + 1])
        dzz = np.array([-1j * np.exp(-1j * g), 1j * np.exp(1j * g), 1j * np.exp(1j * g),
                        -1j * np.exp(-1j * g)])
        dx = np.array([-np.sin(b), -1j * np.cos(b), -1j * np.cos(b), -np.sin(b)])
        for _ in range(n):
            grad[2 * layer] += np.real(np.sum(np.asarray(cots[k]).reshape(-1) * dzz))
            k += 1
        for _ in range(n):
            grad[2 * layer + 1] += np.real(np.sum(np.asarray(cots[k]).reshape(-1) * dx))
            k += 1
    return e, grad
