"""RCCL communicator bootstrap for the sharded state, one process per GPU (no PyTorch).

The native runtime owns the RCCL communicator (C ABI qdc_comm_*).  Rank 0 creates the
128-byte ncclUniqueId and publishes it in a file (written to a temporary name, then renamed, so
a reader never sees a partial id); the other ranks poll for it.  The file name is unique per
launch (QDC_NCCL_ID_FILE, else derived from MASTER_ADDR/MASTER_PORT and the run id that
torchrun or any launcher exports); rank 0 removes it once the communicator exists
(ncclCommInitRank returns only after every rank has joined, i.e. has read it).  Usage, under
any launcher that exports RANK / WORLD_SIZE / LOCAL_RANK (torchrun, mpirun wrappers, a shell
loop):

    from quantum_differentiable_circuit import circuit_class
    from quantum_differentiable_circuit.distributed import Communicator
    comm = Communicator("f32")                 # collective; device = LOCAL_RANK
    c = circuit_class("f32")(30, comm=comm)    # the 2^30 state, 2^(30-g) amplitudes per rank

One process driving all GPUs needs none of this: circuit_class("f32")(30, devices=4).
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
import time
from pathlib import Path

from ._native import check, load


def set_device(index: int):
    hip = C.CDLL("libamdhip64.so")
    err = hip.hipSetDevice(C.c_int(index))
    if err != 0:
        raise RuntimeError(f"hipSetDevice({index}) failed with error {err}")


def default_id_file(world: int) -> Path:
    if os.environ.get("QDC_NCCL_ID_FILE"):
        return Path(os.environ["QDC_NCCL_ID_FILE"])
    tag = "_".join(os.environ.get(k, "x") for k in ("MASTER_ADDR", "MASTER_PORT",
                                                     "TORCHELASTIC_RUN_ID"))
    tag = "".join(ch if ch.isalnum() else "_" for ch in tag)
    return Path(tempfile.gettempdir()) / f"qdc_nccl_id_{tag}_w{world}"


def exchange_id(rank: int, path: Path, make_id, timeout: float = 300.0) -> bytes:
    """Rank 0 publishes make_id()'s 128 bytes at `path` (temporary name + rename: never seen
    partial); every other rank polls for it."""
    path = Path(path)
    if rank == 0:
        raw = make_id()
        tmp = path.with_name(path.name + f".tmp{os.getpid()}")
        tmp.write_bytes(raw)
        os.replace(tmp, path)
        return raw
    t0 = time.monotonic()
    while True:
        try:
            raw = path.read_bytes()
            if len(raw) == 128:
                return raw
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no RCCL id at {path} after {timeout} s")
        time.sleep(0.05)


class Communicator:
    def __init__(self, precision: str = "f32", rank: int | None = None, world: int | None = None,
                 device: int | None = None, id_file: str | os.PathLike | None = None,
                 timeout: float = 300.0):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else int(world)
        if self.world < 1 or self.world & (self.world - 1):
            raise ValueError("the number of ranks must be a power of two")
        self.precision = precision
        self._lib = load(precision)
        set_device(int(os.environ.get("LOCAL_RANK", self.rank)) if device is None else device)
        path = Path(id_file) if id_file else default_id_file(self.world)

        def make_id():
            uid = C.create_string_buffer(128)
            check(self._lib.qdc_comm_unique_id(uid))
            return uid.raw

        raw = exchange_id(self.rank, path, make_id, timeout)
        h = C.c_void_p()
        check(self._lib.qdc_comm_init(C.byref(h), self.rank, self.world, raw))
        self.handle = h
        if self.rank == 0:
            try:
                path.unlink()
            except FileNotFoundError:
                pass

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self._lib.qdc_comm_free(h)
            self.handle = None
