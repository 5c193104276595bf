import os, sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/differentiable-quantum-circuit-cuda_amd')
from oracle import oracle as O
import quantum_differentiable_circuit as q
n, layers = int(sys.argv[1]), int(sys.argv[2])
ins, const, var, pert = O.autodiff_circuit(n, layers, seed=42)
o = O.OracleCircuit(n)
for k, p in ins: o.add(k, *p)
dens = o.forward(const, var)
_, cots = O.tsallis_loss_and_cotangents(dens)
cots = [np.ascontiguousarray(c.conj()) for c in cots]
grads = o.backward(cots, const, var)
def nr(a, b):
    a = np.concatenate([np.asarray(x).reshape(-1) for x in a]); b = np.concatenate([np.asarray(x).reshape(-1) for x in b])
    return np.abs(a-b).max()/np.abs(b).max()
for env in ({'QDC_FUSE': '0'}, {'QDC_FUSE': '1', 'QDC_FUSE_MEAS': '0'}, {'QDC_FUSE': '1', 'QDC_FUSE_MEAS': '1'}):
    os.environ.update(env)
    c = q.circuit_class('f64')(n)
    for k, p in ins: c._push(k, *p)
    d = c.forward(const, var)
    g = c.backward(cots, const, var)
    # per-density error
    errs = [np.abs(a-b).max() for a, b in zip(d, dens)]
    gerrs = [np.abs(a-b).max() for a, b in zip(g, grads)]
    print(env, 'dens', '%.2e' % nr(d, dens), 'first bad dens', next((i for i, e in enumerate(errs) if e > 1e-9), None),
          'grads', '%.2e' % nr(g, grads), 'first bad grad', next((i for i, e in enumerate(gerrs) if e > 1e-9), None), flush=True)
    del c
