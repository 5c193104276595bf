"""RCCL communicator bootstrap for the sharded state, one process per GPU (no PyTorch).

The native runtime owns the RCCL communicator (C ABI qdc_comm_*).  Rank 0 creates the
128-byte ncclUniqueId and publishes it in a file (written to a temporary name, then renamed, so
a reader never sees a partial id); the other ranks poll for it.  The file is bound to this
launch twice over: its name carries MASTER_ADDR/MASTER_PORT, the launcher's run id and the
launcher's process id (the ranks' common parent under torchrun or mpirun), and its contents
carry rank 0's start time, host and process id: a reader accepts an id only when that start
time is within `skew` seconds of its own start and, on the same host, that rank 0 is still
alive — so an id left behind by an earlier launch that died before rank 0 removed it (same
name: a shell loop relaunching from one parent) is never taken for this launch's.  rank 0
removes any earlier file before it publishes, and removes its own
once the communicator exists (ncclCommInitRank returns only after every rank has joined, i.e.
has read it).  The file lives in the node's temporary directory: this bootstrap is single-node
(QDC_NCCL_ID_FILE may name a shared path for more).  Usage, under any launcher that exports
RANK / WORLD_SIZE / LOCAL_RANK (torchrun, mpirun wrappers, a shell loop):

    from quantum_differentiable_circuit import circuit_class
    from quantum_differentiable_circuit.distributed import Communicator
    comm = Communicator("f32")                 # collective; device = LOCAL_RANK
    c = circuit_class("f32")(30, comm=comm)    # the 2^30 state, 2^(30-g) amplitudes per rank

One process driving all GPUs needs none of this: circuit_class("f32")(30, devices=4).
"""
from __future__ import annotations

import ctypes as C
import os
import struct
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
    return Path(tempfile.gettempdir()) / f"qdc_nccl_id_{tag}_p{os.getppid()}_w{world}"


def process_start_time() -> float:
    """Wall-clock start of this process (Linux /proc; else now)."""
    try:
        ticks = int(Path("/proc/self/stat").read_text().rsplit(")", 1)[1].split()[19])
        boot = next(float(l.split()[1]) for l in Path("/proc/stat").read_text().splitlines()
                    if l.startswith("btime"))
        return boot + ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError, StopIteration):
        return time.time()


_ID_LEN = 128
# after the id: rank 0's start time, process id, PID-namespace identity and host name
_FMT = "<dqQ64s"


def pid_namespace() -> int:
    """Identity of this process's PID namespace (the inode of /proc/self/ns/pid; 0 if unknown).
    Ranks may share a host name (a shared UTS namespace) but not a PID namespace (containers
    with a mounted /tmp): rank 0's pid is then meaningless to them."""
    try:
        return os.stat("/proc/self/ns/pid").st_ino
    except OSError:
        return 0


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:  # another user's process: exists
        return True
    return True


def exchange_id(rank: int, path: Path, make_id, timeout: float = 300.0, skew: float = 120.0,
                start: float | None = None) -> bytes:
    """Rank 0 publishes make_id()'s 128 bytes, its start time, pid and host at `path` (temporary
    name + rename: never seen partial); every other rank polls for a file whose rank-0 start
    time is within `skew` s of its own start (ranks of one launch start together; a stale file
    of an earlier launch is older) and whose rank 0, if on this host, is alive (a launch that
    died left its file behind)."""
    path = Path(path)
    start = process_start_time() if start is None else start
    host = os.uname().nodename.encode()[:64]
    ns = pid_namespace()
    if rank == 0:
        try:
            path.unlink()  # an earlier launch's file: gone before this launch's id appears
        except FileNotFoundError:
            pass
        raw = make_id()
        tmp = path.with_name(path.name + f".tmp{os.getpid()}")
        tmp.write_bytes(raw + struct.pack(_FMT, start, os.getpid(), ns, host))
        os.replace(tmp, path)
        return raw
    t0 = time.monotonic()
    while True:
        try:
            data = path.read_bytes()
            if len(data) == _ID_LEN + struct.calcsize(_FMT):
                t_root, pid, ns_root, h = struct.unpack(_FMT, data[_ID_LEN:])
                # rank 0's pid is checked on the same host in the same PID namespace; when
                # either namespace is unknown (0), the host name alone decides (the old rule),
                # so only namespaces known to differ skip the liveness check
                known = ns != 0 and ns_root != 0
                same = h.rstrip(b"\0") == host and (ns_root == ns or not known)
                live = not same or _alive(pid)
                if abs(t_root - start) <= skew and live:
                    return data[:_ID_LEN]
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no RCCL id of this launch at {path} after {timeout} s")
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

    # host-value collectives over the same RCCL communicator (qdc_comm_allreduce)
    def allreduce(self, values, op: str = "sum"):
        vals = [float(v) for v in values]
        arr = (C.c_double * max(len(vals), 1))(*vals)
        check(self._lib.qdc_comm_allreduce(self.handle, arr, len(vals), 0 if op == "sum" else 1))
        return [arr[i] for i in range(len(vals))]

    def barrier(self):
        check(self._lib.qdc_comm_allreduce(self.handle, None, 0, 0))

    def max(self, x: float) -> float:
        return self.allreduce([x], "max")[0]

    def sum(self, x: float) -> float:
        return self.allreduce([x], "sum")[0]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self._lib.qdc_comm_free(h)
            self.handle = None
