# can two RCCL ranks share one GPU? (probe for testing the RCCL transport on a 1-GPU box)
import os, sys
sys.path.insert(0, "differentiable-quantum-circuit-cuda_amd"); sys.path.insert(0, ".")
import numpy as np
import torch.distributed as dist
dist.init_process_group("gloo")
rank = dist.get_rank()
from quantum_differentiable_circuit.distributed import Communicator
import quantum_differentiable_circuit as q
try:
    comm = Communicator("f64", device=0)
    c = q.circuit_class("f64")(10, comm=comm)
    c.add_q1_var_gate(9); c.get_q1_dens_op_with_grad(9)
    d = c.forward([], [np.array([0, 1, 1, 0], np.complex128)])
    print(rank, "OK", d[0].real.round(3).tolist(), flush=True)
except BaseException as e:
    print(rank, "FAIL", type(e).__name__, str(e)[:300], flush=True)
