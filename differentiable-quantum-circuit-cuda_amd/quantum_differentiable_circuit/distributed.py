"""RCCL communicator bootstrap for the sharded state (one process per GPU).

The native runtime owns the RCCL communicator (C ABI qdc_comm_*); torch.distributed is only
the plumbing that ships rank 0's 128-byte ncclUniqueId to the other ranks (any backend, gloo
is enough).  Usage, under `python -m torch.distributed.run --nproc-per-node N ...`:

    import torch.distributed as dist
    from quantum_differentiable_circuit import circuit_class
    from quantum_differentiable_circuit.distributed import Communicator
    dist.init_process_group("gloo")
    comm = Communicator("f32")                 # collective; device = LOCAL_RANK
    c = circuit_class("f32")(30, comm=comm)    # the 2^30 state, 2^(30-g) amplitudes per rank
"""
from __future__ import annotations

import ctypes as C
import os

from ._native import check, load


def set_device(index: int):
    hip = C.CDLL("libamdhip64.so")
    err = hip.hipSetDevice(C.c_int(index))
    if err != 0:
        raise RuntimeError(f"hipSetDevice({index}) failed with error {err}")


class Communicator:
    def __init__(self, precision: str = "f32", device: int | None = None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("initialise torch.distributed first (the id bootstrap uses it)")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        if self.world & (self.world - 1):
            raise ValueError("the number of ranks must be a power of two")
        self.precision = precision
        self._lib = load(precision)
        set_device(int(os.environ.get("LOCAL_RANK", self.rank)) if device is None else device)
        uid = C.create_string_buffer(128)
        if self.rank == 0:
            check(self._lib.qdc_comm_unique_id(uid))
        box = [uid.raw if self.rank == 0 else None]
        dist.broadcast_object_list(box, 0)
        h = C.c_void_p()
        check(self._lib.qdc_comm_init(C.byref(h), self.rank, self.world, box[0]))
        self.handle = h

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self._lib.qdc_comm_free(h)
            self.handle = None
