# Can two RCCL ranks share one GPU?  If so, the one-process-per-GPU RCCL transport (pack +
# ncclAllToAll remaps, ncclAllReduce of densities / gradients) runs on a 1-GPU box: a random
# circuit sharded over 2 ranks, forward + backward, against the same circuit unsharded.
# Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ...
import os, sys
sys.path.insert(0, "differentiable-quantum-circuit-cuda_amd"); sys.path.insert(0, ".")
import numpy as np
import torch.distributed as dist
dist.init_process_group("gloo")
rank = dist.get_rank()
from quantum_differentiable_circuit.distributed import Communicator
from quantum_differentiable_circuit import workloads as W
import quantum_differentiable_circuit as q
prec = os.environ.get("PROBE_PREC", "f64")
n = 12
ins, const, var = W.random_circuit(n, 80, seed=9, density_every=20)
dt = np.complex128 if prec == "f64" else np.complex64
const = [np.ascontiguousarray(g, dt) for g in const]
var = [np.ascontiguousarray(g, dt) for g in var]


def run(c):
    for kind, pos in ins:
        c._push(kind, *pos)
    d = c.forward(const, var)
    cots = [np.ascontiguousarray(np.eye(x.shape[0]), dt) for x in d]
    g = c.backward(cots, const, var)
    return d, g


try:
    comm = Communicator(prec, device=0)
    d, g = run(q.circuit_class(prec)(n, comm=comm))
    print(rank, "RCCL sharded run OK", flush=True)
    if rank == 0:
        d0, g0 = run(q.circuit_class(prec)(n))
        dd = max(float(np.abs(a - b).max()) for a, b in zip(d, d0))
        gg = max(float(np.abs(a - b).max()) for a, b in zip(g, g0))
        print(f"max |sharded - single| densities {dd:.3e} gradients {gg:.3e}", flush=True)
except BaseException as e:
    print(rank, "FAIL", type(e).__name__, str(e)[:400], flush=True)
dist.barrier()
