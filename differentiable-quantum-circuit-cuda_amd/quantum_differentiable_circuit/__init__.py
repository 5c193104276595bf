"""quantum_differentiable_circuit — drop-in for the reference's PyO3 module of the same name
(``src/circuit.rs:432-436``), backed by the HIP/gfx950 runtime in ``libqdc_{f32,f64}.so``.

``Circuit`` reproduces ``#[pyclass] Circuit`` (``src/circuit.rs:86-430``) method for method:
the builders, ``run``, ``forward`` and ``backward``, their argument order, their outputs
(lists of 2-D density matrices / 1-D gate gradients) and their panic messages.  Like the
reference there is one precision per library; the module-level ``Circuit`` uses the precision
named by ``QDC_PRECISION`` (``f32`` default, or ``f64``), and ``Circuit32`` / ``Circuit64`` pin
one explicitly.  Input arrays must have the build's dtype (complex64 / complex128), as PyO3's
``PyReadonlyArray1<Complex>`` extraction demands.

``QuantizedTensor`` and the ``get_q*_grad`` / ``data_transfer`` helpers mirror
``src/quantized_tensor.rs:54-238`` over the 18-function C ABI, so the parity tests can follow
the reference's own unit tests (``quantized_tensor.rs:400-609``).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np

from .common_gates import get_cnot, get_hadamard  # noqa: E402  (common_gates.rs)
from ._native import (PanicException, KernelStat, PlanOp, check, default_precision, load,
                      ptr, PRECISIONS)

__all__ = ["Circuit", "Circuit32", "Circuit64", "QuantizedTensor", "PanicException",
           "get_q1_grad", "get_q2_grad", "get_q2_grad_diag", "data_transfer", "circuit_class",
           "plan", "unpermute", "get_hadamard", "get_cnot"]

# enum Instruction order (src/circuit.rs:53-68) == enum qdc_kind (include/qdc/circuit.h)
(CONST_Q2, VAR_Q2, CONST_Q2_NONU, VAR_Q2_NONU, CONST_Q2_DIAG, VAR_Q2_DIAG, CONST_Q1,
 CONST_Q1_NONU, VAR_Q1, VAR_Q1_NONU, Q2_DENSITY, Q1_DENSITY, DIFF_Q2_DENSITY,
 DIFF_Q1_DENSITY) = range(14)
MODE_RUN, MODE_FORWARD = 0, 1


def _array1(x, dtype, what):
    """PyReadonlyArray1<Complex> extraction: an ndarray of exactly this dtype and ndim 1."""
    if not isinstance(x, np.ndarray) or x.dtype != dtype or x.ndim != 1:
        raise TypeError(f"argument '{what}': expected a 1-D numpy array of {np.dtype(dtype)}")
    return x


def _array2(x, dtype, what):
    if not isinstance(x, np.ndarray) or x.dtype != dtype or x.ndim != 2:
        raise TypeError(f"argument '{what}': expected a 2-D numpy array of {np.dtype(dtype)}")
    return x


def _flat_gates(gates, dtype, what):
    """_array1 on every gate, then _flatten, in one pass over the list (a C2 step passes ~1100
    gates twice: the checks, not the copy, dominate); any failed check takes the per-array
    path for the reference's exact error."""
    sizes = []
    add = sizes.append
    for g in gates:
        if g.__class__ is not np.ndarray or g.dtype != dtype or g.ndim != 1 or \
                not g.flags.c_contiguous:
            return _flatten([_array1(x, dtype, what) for x in gates], dtype, what,
                            "Gate is not contiguous.")
        add(g.size)
    if not sizes:
        return np.zeros(1, dtype), np.zeros(1, np.uintp)
    return np.concatenate(gates), np.array(sizes, dtype=np.uintp)


def _flatten(arrays, dtype, what, msg):
    """Concatenate host buffers for the C ABI; as_slice() panics on non-contiguous input."""
    lens = np.fromiter((a.size for a in arrays), dtype=np.uintp, count=len(arrays))
    for a in arrays:
        if not a.flags.c_contiguous:
            raise PanicException(msg)
    flat = np.concatenate([a.reshape(-1) for a in arrays]) if arrays else np.zeros(1, dtype)
    return np.ascontiguousarray(flat, dtype=dtype), lens if len(arrays) else np.zeros(1, np.uintp)


class _CircuitBase:
    _precision = "f32"

    def __init__(self, qubits_number: int, comm=None, local_shards: int | None = None,
                 devices=None):
        """Sharding (none of it exists in the reference, which is single-GPU):
        `comm` (a `distributed.Communicator`) shards the state over its ranks, one GPU per
        process; `devices` (a count or a list of device indices) shards it over several GPUs
        driven by this one process (ncclCommInitAll; a repeated device keeps every shard on it,
        each on its own stream); `local_shards=G` keeps G shards on this GPU and one stream
        (same data path, device copies instead of RCCL)."""
        self._lib = load(self._precision)
        self._dtype = np.dtype(PRECISIONS[self._precision])
        h = C.c_void_p()
        if comm is not None:
            if comm.precision != self._precision:
                raise ValueError("communicator was created for the other precision library")
            check(self._lib.qdc_circuit_new_sharded(C.byref(h), int(qubits_number), comm.handle))
        elif devices is not None:
            devs = list(range(devices)) if isinstance(devices, int) else [int(d) for d in devices]
            arr = (C.c_int * len(devs))(*devs)
            check(self._lib.qdc_circuit_new_devices(C.byref(h), int(qubits_number), len(devs), arr))
        elif local_shards is not None:
            check(self._lib.qdc_circuit_new_local_shards(C.byref(h), int(qubits_number),
                                                         int(local_shards)))
        else:
            check(self._lib.qdc_circuit_new(C.byref(h), int(qubits_number)))
        self._comm = comm  # keep the communicator alive as long as the circuit
        self._h = h
        self._n = int(qubits_number)
        self._kinds = []  # instruction kinds, for splitting the flat outputs

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.qdc_circuit_free(h)
            self._h = None

    @property
    def qubits_number(self) -> int:
        return self._n

    @property
    def dtype(self):
        return self._dtype

    # --- circuit.rs:104-106 -----------------------------------------------------------
    def set_state_from_vector(self, vector: np.ndarray) -> None:
        v = _array1(vector, self._dtype, "vector")
        if not v.flags.c_contiguous:
            raise PanicException("called `Option::unwrap()` on a `None` value")
        check(self._lib.qdc_circuit_set_state_from_vector(self._h, ptr(v), v.size))

    # --- builders, circuit.rs:108-162 -------------------------------------------------
    def _push(self, kind, a, b=0):
        if a < 0 or b < 0:
            raise OverflowError("can't convert negative int to unsigned")
        check(self._lib.qdc_circuit_push(self._h, kind, int(a), int(b)))
        self._kinds.append(kind)

    def add_q2_const_gate(self, pos2: int, pos1: int): self._push(CONST_Q2, pos2, pos1)
    def add_q2_const_gate_diag(self, pos2: int, pos1: int): self._push(CONST_Q2_DIAG, pos2, pos1)
    def add_q2_const_gate_nonu(self, pos2: int, pos1: int): self._push(CONST_Q2_NONU, pos2, pos1)
    def add_q2_var_gate(self, pos2: int, pos1: int): self._push(VAR_Q2, pos2, pos1)
    def add_q2_var_gate_diag(self, pos2: int, pos1: int): self._push(VAR_Q2_DIAG, pos2, pos1)
    def add_q2_var_gate_nonu(self, pos2: int, pos1: int): self._push(VAR_Q2_NONU, pos2, pos1)
    def add_q1_const_gate(self, pos: int): self._push(CONST_Q1, pos)
    def add_q1_const_gate_nonu(self, pos: int): self._push(CONST_Q1_NONU, pos)
    def add_q1_var_gate(self, pos: int): self._push(VAR_Q1, pos)
    def add_q1_var_gate_nonu(self, pos: int): self._push(VAR_Q1_NONU, pos)
    def get_q2_dens_op(self, pos2: int, pos1: int): self._push(Q2_DENSITY, pos2, pos1)
    def get_q1_dens_op(self, pos: int): self._push(Q1_DENSITY, pos)
    def get_q2_dens_op_with_grad(self, pos2: int, pos1: int): self._push(DIFF_Q2_DENSITY, pos2, pos1)
    def get_q1_dens_op_with_grad(self, pos: int): self._push(DIFF_Q1_DENSITY, pos)

    def __len__(self):
        return int(self._lib.qdc_circuit_len(self._h))

    # --- execution ---------------------------------------------------------------------
    def _gates(self, gates: Sequence[np.ndarray], what: str):
        return _flat_gates(gates, self._dtype, what)

    def run(self, const_gates: List[np.ndarray], var_gates: List[np.ndarray]) -> List[np.ndarray]:
        """circuit.rs:164-212: every density matrix, in instruction order."""
        return self._exec(MODE_RUN, const_gates, var_gates)

    def forward(self, const_gates: List[np.ndarray], var_gates: List[np.ndarray]) -> List[np.ndarray]:
        """circuit.rs:214-264: the Diff* density matrices, in instruction order."""
        return self._exec(MODE_FORWARD, const_gates, var_gates)

    def _exec(self, mode, const_gates, var_gates):
        cf, cl = self._gates(const_gates, "const_gates")
        vf, vl = self._gates(var_gates, "var_gates")
        size = int(self._lib.qdc_circuit_output_size(self._h, mode))
        out = np.empty(max(size, 1), dtype=self._dtype)
        check(self._lib.qdc_circuit_execute(self._h, mode, ptr(cf), ptr(cl), len(const_gates),
                                             ptr(vf), ptr(vl), len(var_gates), ptr(out)))
        res, o = [], 0
        for is_q1 in self._out_kinds(mode):
            k = 2 if is_q1 else 4
            res.append(out[o:o + k * k].reshape(k, k).copy())
            o += k * k
        assert o == size
        return res

    def backward(self, grads_wrt_density: List[np.ndarray], const_gates: List[np.ndarray],
                 var_gates: List[np.ndarray]) -> List[np.ndarray]:
        """circuit.rs:266-429: gradients of the variable gates, forward order."""
        dens = [_array2(g, self._dtype, "grads_wrt_density") for g in grads_wrt_density]
        df, dl = _flatten(dens, self._dtype, "grads_wrt_density", "Gradient is not contiguous.")
        cf, cl = self._gates(const_gates, "const_gates")
        vf, vl = self._gates(var_gates, "var_gates")
        size = int(self._lib.qdc_circuit_grad_size(self._h))
        out = np.empty(max(size, 1), dtype=self._dtype)
        check(self._lib.qdc_circuit_backward(self._h, ptr(df), ptr(dl), len(dens), ptr(cf),
                                              ptr(cl), len(const_gates), ptr(vf), ptr(vl),
                                              len(var_gates), ptr(out)))
        # one array per gate that owns its data, as the reference returns (circuit.rs:429)
        return [out[sl].copy() for sl in self._grad_slices()]

    # --- instruction metadata (kept on the Python side for output splitting) -----------
    def _out_kinds(self, mode):
        return [k in (Q1_DENSITY, DIFF_Q1_DENSITY) for k in self._kinds
                if k in (DIFF_Q1_DENSITY, DIFF_Q2_DENSITY)
                or (mode == MODE_RUN and k in (Q1_DENSITY, Q2_DENSITY))]

    def _grad_slices(self):
        """Slices of the gradient buffer per variable gate (cached until the next push)."""
        key = len(self._kinds)
        if getattr(self, "_gs_key", None) != key:
            sl, o = [], 0
            for w in self._var_widths():
                sl.append(slice(o, o + w))
                o += w
            self._gs, self._gs_key = sl, key
        return self._gs

    def _var_widths(self):
        return [16 if k in (VAR_Q2, VAR_Q2_NONU) else 4 for k in self._kinds
                if k in (VAR_Q1, VAR_Q1_NONU, VAR_Q2, VAR_Q2_NONU, VAR_Q2_DIAG)]

    # --- extras (not in the reference's Python surface) --------------------------------
    def layout(self):
        """(phys, world, first_rank, local_shards): phys[q] = physical bit of logical qubit q."""
        phys = (C.c_uint * self._n)()
        w, r, ls = C.c_int(), C.c_int(), C.c_int()
        check(self._lib.qdc_circuit_layout(self._h, phys, C.byref(w), C.byref(r), C.byref(ls)))
        return list(phys), w.value, r.value, ls.value

    def get_shard(self, which: int = 0, shard: int = 0) -> np.ndarray:
        phys, world, _, _ = self.layout()
        out = np.empty(1 << (self._n - (world.bit_length() - 1)), dtype=self._dtype)
        check(self._lib.qdc_circuit_get_shard(self._h, which, shard, ptr(out), out.size))
        return out

    def get_range(self, which: int, offset: int, count: int, shard: int = 0) -> np.ndarray:
        """`count` amplitudes of a local shard from `offset`, in PHYSICAL order (see layout())."""
        out = np.empty(count, dtype=self._dtype)
        check(self._lib.qdc_circuit_get_range(self._h, which, shard, offset, ptr(out), count))
        return out

    def get_state(self, which: int = 0) -> np.ndarray:
        """Copy of the forward (0), initial (1) or backward (2) state in logical qubit order.
        Sharded over processes: collective — the shards are gathered over the circuit's own
        RCCL communicator (qdc_circuit_gather_state)."""
        phys, world, rank0, nlocal = self.layout()
        out = np.empty(1 << self._n, dtype=self._dtype)
        if world == 1:
            # (logical order: the library undoes a permuted single-device layout)
            check(self._lib.qdc_circuit_get_state(self._h, which, ptr(out), out.size))
            return out
        check(self._lib.qdc_circuit_gather_state(self._h, which, ptr(out), out.size))
        if which == 1:
            phys = list(range(self._n))  # `initial` is always in the identity layout
        return unpermute(out, phys)

    def synchronize(self):
        check(self._lib.qdc_circuit_sync(self._h))

    def profile(self, on: bool):
        check(self._lib.qdc_circuit_profile(self._h, 1 if on else 0))

    def profile_collect(self):
        cap = 64
        buf = (KernelStat * cap)()
        k = int(self._lib.qdc_circuit_profile_collect(self._h, buf, cap))
        return {buf[i].name.decode(): {"launches": int(buf[i].launches),
                                        "total_ms": float(buf[i].total_ms),
                                        "algo_bytes": float(buf[i].algo_bytes),
                                        "algo_flops": float(buf[i].algo_flops)}
                for i in range(min(k, cap))}

    def host_times(self, reset=False):
        """Host milliseconds of this circuit's calls since the last reset (qdc_circuit_host_times):
        {"forward" | "backward": {"calls", "setup", "schedule", "build", "launch", "finish"}}
        ("forward" includes run calls)."""
        buf = (C.c_double * 12)()
        self._lib.qdc_circuit_host_times(self._h, buf, 12, 1 if reset else 0)
        keys = ("calls", "setup", "schedule", "build", "launch", "finish")
        return {d: {k: buf[6 * i + j] for j, k in enumerate(keys)}
                for i, d in enumerate(("forward", "backward"))}


def primitives_sync(precision=None):
    """Wait for the primitives' stream (qdc_abi_sync, include/qdc/dense.h)."""
    check(load(precision or default_precision()).qdc_abi_sync())


def primitives_profile(on: bool, precision=None):
    """Per-launch HIP-event profiling of the primitives' stream (qdc_abi_profile)."""
    check(load(precision or default_precision()).qdc_abi_profile(1 if on else 0))


def primitives_profile_collect(precision=None):
    lib = load(precision or default_precision())
    cap = 64
    buf = (KernelStat * cap)()
    k = int(lib.qdc_abi_profile_collect(buf, cap))
    return {buf[i].name.decode(): {"launches": int(buf[i].launches),
                                    "total_ms": float(buf[i].total_ms),
                                    "algo_bytes": float(buf[i].algo_bytes),
                                    "algo_flops": float(buf[i].algo_flops)}
            for i in range(min(k, cap))}


class Circuit32(_CircuitBase):
    """Single-precision build (complex64), like `maturin develop --release`."""
    _precision = "f32"


class Circuit64(_CircuitBase):
    """Double-precision build (complex128), like `maturin develop --features "f64"`."""
    _precision = "f64"


def circuit_class(precision: str | None = None):
    p = precision or default_precision()
    return Circuit64 if p == "f64" else Circuit32


Circuit = circuit_class()


def unpermute(physical: np.ndarray, phys) -> np.ndarray:
    """Reorder a state stored in a physical layout (rank bits on top) into logical qubit order."""
    n = len(phys)
    t = physical.reshape((2,) * n)  # axis k <-> physical bit n-1-k
    axes = [n - 1 - phys[n - 1 - k] for k in range(n)]  # logical axis k = qubit n-1-k
    return np.ascontiguousarray(t.transpose(axes)).reshape(-1)


def plan(qubits_number, world, instructions, mode, start_phys=None, precision=None):
    """The sharding planner of the native runtime (qdc_plan, host only): returns
    (ops, end_phys); ops are dicts {"type": "op"|"remap", ...}.  mode: 0 run, 1 forward,
    2 backward, 3 mirrored forward (ops keep both directions' order relations: its plan run in
    reverse, every remap undone, is the backward's).  `instructions` = [(kind, pos2[, pos1])]."""
    lib = load(precision or default_precision())
    m = len(instructions)
    kinds = (C.c_int * m)(*[int(i[0]) for i in instructions])
    a = (C.c_uint * m)(*[int(i[1]) for i in instructions])
    b = (C.c_uint * m)(*[int(i[2]) if len(i) > 2 else 0 for i in instructions])
    sp = (C.c_uint * qubits_number)(*start_phys) if start_phys is not None else None
    cap = 4 * m + 16
    out = (PlanOp * cap)()
    end = (C.c_uint * qubits_number)()
    k = int(lib.qdc_plan(qubits_number, world, kinds, a, b, m, mode, sp, out, cap, end))
    if k == 0 and m > 0:
        raise ValueError("planner rejected the configuration")
    ops = []
    for i in range(min(k, cap)):
        o = out[i]
        if o.type == 0:
            ops.append({"type": "op", "instr": o.instr, "pos2": o.pos2, "pos1": o.pos1})
        else:
            ops.append({"type": "remap", "victims": list(o.victims[:o.nvictims]), "pack": bool(o.pack)})
    return ops, list(end)


def fusion_schedule(qubits_number, instructions, mode, fwd_sens=None, precision=None,
                    lcmin=0, max_ops=0):
    """The fused-pass scheduler of the native runtime (qdc_fusion_schedule, host only) on the
    unsharded plan of `instructions` = [(kind, pos2[, pos1])]; mode 0 run, 1 forward,
    2 backward.  Returns (plan, items): plan = the dicts of `plan()`, items = execution-ordered
    [{"type": 0 single | 1 remap | 2 fused, "lc", "h", "hb", "stages": [[plan index, ...]]}]."""
    lib = load(precision or default_precision())
    m = len(instructions)
    kinds_l = [int(i[0]) for i in instructions]
    kinds = (C.c_int * m)(*kinds_l)
    a = (C.c_uint * m)(*[int(i[1]) for i in instructions])
    b = (C.c_uint * m)(*[int(i[2]) if len(i) > 2 else 0 for i in instructions])
    cap = 4 * m + 16
    raw = (PlanOp * cap)()
    k = int(lib.qdc_plan(qubits_number, 1, kinds, a, b, m, mode, None, raw, cap, None))
    ops = [{"type": "op", "instr": raw[i].instr, "pos2": raw[i].pos2, "pos1": raw[i].pos1}
           for i in range(k)]
    first_inject = 2**64 - 1
    if mode == 2:
        for i, o in enumerate(ops):
            if kinds_l[o["instr"]] in (12, 13):  # DiffQ2Density, DiffQ1Density
                first_inject = i
                break
    sens = (C.c_ubyte * m)(*[1 if x else 0 for x in (fwd_sens or [0] * m)])
    icap, scap, ocap = k + 1, k + 1, k + 1
    info = (C.c_uint * (12 * icap))()
    slen = (C.c_uint * scap)()
    order = (C.c_uint * ocap)()
    n_items = int(lib.qdc_fusion_schedule(qubits_number, 1 if mode == 2 else 0, first_inject,
                                          kinds, sens, m, raw, k, lcmin, max_ops, info, icap,
                                          slen, scap, order, ocap))
    if n_items == 2**64 - 1:
        raise RuntimeError("fusion schedule output capacity exceeded")
    items, si, oi = [], 0, 0
    for i in range(n_items):
        t, nst, lc, h = info[12 * i], info[12 * i + 1], info[12 * i + 2], info[12 * i + 3]
        stages = []
        for _ in range(nst):
            stages.append([int(order[oi + j]) for j in range(slen[si])])
            oi += slen[si]
            si += 1
        items.append({"type": int(t), "lc": int(lc), "h": int(h),
                      "hb": [int(info[12 * i + 4 + j]) for j in range(min(h, 8))],
                      "stages": stages})
    return ops, items


def rq_plan(tile_bits, stages, deps=None, precision=None, slots=4):
    """The register-layout plan of a register-resident pass (qdc_rq_plan, host only).
    stages = [(kind 0 one-qubit | 1 two-qubit | 2 diagonal, t1, t2)] in tile bits; deps[i] =
    bit mask of the earlier stages stage i must follow; `slots` register slots (4, or 5 for the
    one-wave two-state f32 kernel).  Returns (load, steps, store): the load / store layouts'
    slots and [{"relayout": bool, "stage": i, "case": c, "slots": [slots]}] (two-qubit case
    8 * slot(t1) + slot(t2))."""
    lib = load(precision or default_precision())
    n = len(stages)
    kinds = (C.c_uint * max(n, 1))(*[int(s[0]) for s in stages])
    t1 = (C.c_uint * max(n, 1))(*[int(s[1]) for s in stages])
    t2 = (C.c_uint * max(n, 1))(*[int(s[2]) for s in stages])
    dp = (C.c_ulonglong * max(n, 1))(*[int(d) for d in (deps or [0] * n)])
    cap = 2 * n + 4
    out = (C.c_uint * (8 * cap))()
    k = int(lib.qdc_rq_plan(tile_bits, slots, kinds, t1, t2, dp, n, out, cap))
    if k == 2**64 - 1:
        raise RuntimeError("rq plan output capacity exceeded")
    rows = [[int(out[8 * i + j]) for j in range(8)] for i in range(k)]
    steps = [{"relayout": r[0] == 1, "stage": r[1], "case": r[2], "slots": r[3:3 + slots]}
             for r in rows[1:-1]]
    return rows[0][3:3 + slots], steps, rows[-1][3:3 + slots]


def spec_selftest(tile_bits, stages, deps=None, precision="f32"):
    """Compile the specialized kernel of a pass (host only: the runtime's generator and hipcc,
    qdc_spec_selftest): f32 tile_bits 11, a five-slot two-state reverse pass; 12, a four-slot
    one-state forward pass; f64 10 two-state, 11 one-state.  stages as for rq_plan.  Returns
    (kernel name, code object path); raises RuntimeError with the runtime's message."""
    lib = load(precision)
    n = len(stages)
    kinds = (C.c_uint * n)(*[int(s[0]) for s in stages])
    t1 = (C.c_uint * n)(*[int(s[1]) for s in stages])
    t2 = (C.c_uint * n)(*[int(s[2]) for s in stages])
    dp = (C.c_ulonglong * n)(*[int(d) for d in (deps or [0] * n)])
    out = C.create_string_buffer(1024)
    err = lib.qdc_spec_selftest(tile_bits, kinds, t1, t2, dp, n, out, 1024)
    if err:
        raise RuntimeError(err.decode())
    raw = out.raw
    name = raw.split(b"\0", 1)[0].decode()
    path = raw[len(name) + 1:].split(b"\0", 1)[0].decode()
    return name, path


def spec_selftest_batch(tile_bits, programs, precision="f32"):
    """spec_selftest for several pass programs [(stages, deps), ...] compiled in one call of the
    kernel cache (qdc_spec_selftest_batch), as a circuit call compiles its missing kernels.
    Returns the kernel names."""
    lib = load(precision)
    counts = (C.c_size_t * len(programs))(*[len(st) for st, _ in programs])
    flat = [s for st, _ in programs for s in st]
    dflat = [int(d) for st, dp in programs for d in (dp or [0] * len(st))]
    n = len(flat)
    kinds = (C.c_uint * n)(*[int(s[0]) for s in flat])
    t1 = (C.c_uint * n)(*[int(s[1]) for s in flat])
    t2 = (C.c_uint * n)(*[int(s[2]) for s in flat])
    dp = (C.c_ulonglong * n)(*dflat)
    out = C.create_string_buffer(64 * len(programs) + 16)
    err = lib.qdc_spec_selftest_batch(tile_bits, counts, len(programs), kinds, t1, t2, dp, out,
                                      len(out))
    if err:
        raise RuntimeError(err.decode())
    return [x.decode() for x in out.raw.split(b"\0")[:len(programs)]]


def jit_stats(precision=None):
    """This process's specialized-kernel cache (qdc_jit_stats): kernels compiled here, kernels
    waited for while another process compiled them, (kernel, device) loads, seconds compiling,
    waiting and in the cache overall, whether specialization is on, launches of specialized
    kernels, and kernels queued for the background compiler."""
    lib = load(precision or default_precision())
    v = (C.c_double * 9)()
    k = int(lib.qdc_jit_stats(v, 9))
    keys = ("compiled", "waited", "loaded", "compile_s", "wait_s", "total_s", "enabled", "launched",
            "queued")
    out = {key: float(v[i]) for i, key in enumerate(keys[:k])}
    for key in ("compiled", "waited", "loaded", "launched", "queued"):
        out[key] = int(out[key])
    out["enabled"] = bool(out["enabled"])
    return out


def jit_wait(timeout_s=3600.0, precision=None):
    """Wait for the background compiler (the specialized kernels of programs with more than
    QDC_SPEC_MAX of them) to drain its queue; returns the kernels still queued."""
    return int(load(precision or default_precision()).qdc_jit_wait(float(timeout_s)))


def precompile(qubits_number, instructions, const_gates, var_gates, grads_wrt_density,
               world=1, precision=None):
    """Compile ahead of time (host only, no GPU) every specialized pass kernel that a forward
    call with these gates, then a backward call with these density cotangents, would launch on a
    circuit of `instructions` = [(kind, pos2[, pos1])] sharded over `world` ranks: the runtime's
    own plans, schedules and pass programs, built by a dry run (qdc_precompile).  The kernels go to
    the cache directory (QDC_JIT_DIR); build() points it at the in-tree prebuilt directory the
    runtime searches after its own cache.  Returns the number of distinct kernels."""
    prec = precision or default_precision()
    lib = load(prec)
    dt = np.dtype(PRECISIONS[prec])
    m = len(instructions)
    kinds = (C.c_int * m)(*[int(i[0]) for i in instructions])
    a = (C.c_uint * m)(*[int(i[1]) for i in instructions])
    b = (C.c_uint * m)(*[int(i[2]) if len(i) > 2 else 0 for i in instructions])
    cf, cl = _flat_gates(const_gates, dt, "const_gates")
    vf, vl = _flat_gates(var_gates, dt, "var_gates")
    dens = [_array2(g, dt, "grads_wrt_density") for g in grads_wrt_density]
    df, dl = _flatten(dens, dt, "grads_wrt_density", "Gradient is not contiguous.")
    count = C.c_size_t(0)
    check(lib.qdc_precompile(int(qubits_number), int(world), kinds, a, b, m, ptr(cf), ptr(cl),
                             len(const_gates), ptr(vf), ptr(vl), len(var_gates), ptr(df), ptr(dl),
                             len(dens), C.byref(count)))
    return int(count.value)


def trace_program(qubits_number, instructions, const_gates, var_gates, grads_wrt_density,
                  world=1, precision=None):
    """Every matrix a forward call then a backward call apply to the forward state, in order, as
    the runtime's own dry run builds them (qdc_trace_program; host only, no GPU): a numpy
    record array with fields dir (0 forward, 1 uncompute), item, q2, q1 (logical qubits; row
    index 2 bit(q2) + bit(q1)), R, diag, mirrored, single and m (R x R in m[:R*R], working
    precision).  For the host drift emulation (tools/drift_emu.py)."""
    prec = precision or default_precision()
    lib = load(prec)
    dt = np.dtype(PRECISIONS[prec])
    rec = np.dtype([("dir", "<u4"), ("item", "<u4"), ("q2", "<u4"), ("q1", "<u4"), ("R", "<u4"),
                    ("diag", "<u4"), ("mirrored", "<u4"), ("single", "<u4"), ("m", dt, 16)])
    m = len(instructions)
    kinds = (C.c_int * m)(*[int(i[0]) for i in instructions])
    a = (C.c_uint * m)(*[int(i[1]) for i in instructions])
    b = (C.c_uint * m)(*[int(i[2]) if len(i) > 2 else 0 for i in instructions])
    cf, cl = _flat_gates(const_gates, dt, "const_gates")
    vf, vl = _flat_gates(var_gates, dt, "var_gates")
    dens = [_array2(g, dt, "grads_wrt_density") for g in grads_wrt_density]
    df, dl = _flatten(dens, dt, "grads_wrt_density", "Gradient is not contiguous.")
    cap = 4 * m + 64
    while True:
        out = np.zeros(cap, dtype=rec)
        cnt = C.c_size_t(0)
        check(lib.qdc_trace_program(int(qubits_number), int(world), kinds, a, b, m, ptr(cf),
                                    ptr(cl), len(const_gates), ptr(vf), ptr(vl), len(var_gates),
                                    ptr(df), ptr(dl), len(dens), ptr(out), cap, C.byref(cnt)))
        if cnt.value <= cap:
            return out[:cnt.value]
        cap = cnt.value


def jit_dir(precision=None):
    """The specialized-kernel cache directory in use; RuntimeError when specialization is off."""
    lib = load(precision or default_precision())
    out = C.create_string_buffer(4096)
    err = lib.qdc_jit_dir(out, 4096)
    if err:
        raise RuntimeError(err.decode())
    return out.value.decode()


def spec_fingerprint(csrc_dir, compiler, defines=None, precision="f32"):
    """(build fingerprint, header hash) a library with `defines` (None: this library's own -D
    switches), compiler identity text `compiler` and the kernel headers of csrc_dir would name
    its specialized kernels with (qdc_spec_fingerprint)."""
    lib = load(precision)
    fp, sh = C.c_ulonglong(), C.c_ulonglong()
    err = lib.qdc_spec_fingerprint(None if defines is None else defines.encode(), compiler.encode(),
                                   str(csrc_dir).encode(), C.byref(fp), C.byref(sh))
    if err:
        raise RuntimeError(err.decode())
    return int(fp.value), int(sh.value)


# ---------------------------------------------------------------------------------------
# QuantizedTensor (src/quantized_tensor.rs:54-238) over the 18-function C ABI
# ---------------------------------------------------------------------------------------
class QuantizedTensor:
    """A device state of 2^n amplitudes owned by this object (RAII like the Rust struct)."""

    def __init__(self, qubits_number: int, precision: str | None = None, _ptr=None):
        self._precision = precision or default_precision()
        self._lib = load(self._precision)
        self.dtype = np.dtype(PRECISIONS[self._precision])
        self.qubits_number = int(qubits_number)
        if _ptr is None:
            p = C.c_void_p()
            check(self._lib.get_state(C.byref(p), self.qubits_number))
            _ptr = p
        self._p = _ptr

    @classmethod
    def new_standard(cls, qubits_number, precision=None):
        t = cls(qubits_number, precision)
        t._lib.set2standard(t._p, t.qubits_number)
        return t

    @classmethod
    def new_from_host(cls, state: np.ndarray, precision=None):
        size = state.size
        if size == 0 or size & (size - 1):
            raise PanicException("State size is not a power of 2.")
        t = cls(size.bit_length() - 1, precision)
        t.set_from_host(state)
        return t

    def __del__(self):
        p = getattr(self, "_p", None)
        if p is not None and p.value:
            check(self._lib.drop_state(p))
            self._p = None

    def _host(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        return a

    def set_from_host(self, state):
        s = self._host(state)
        if s.size != (1 << self.qubits_number):
            raise PanicException("Size of the given state does not match the size of the tensor.")
        check(self._lib.set_from_host(self._p, ptr(s), self.qubits_number))

    def get_cpu_state_copy(self) -> np.ndarray:
        out = np.empty(1 << self.qubits_number, dtype=self.dtype)
        check(self._lib.copy_to_host(self._p, ptr(out), self.qubits_number))
        return out

    def clone(self):
        t = QuantizedTensor(self.qubits_number, self._precision)
        self._lib.copy(self._p, t._p, self.qubits_number)
        return t

    def conj_and_double(self):
        t = QuantizedTensor(self.qubits_number, self._precision)
        self._lib.conj_and_double(self._p, t._p, self.qubits_number)
        return t

    def add(self, other: "QuantizedTensor"):
        if other.qubits_number != self.qubits_number:
            raise PanicException("Tensors have diferent sizes.")
        self._lib.add(other._p, self._p, self.qubits_number)

    def _gate(self, gate, want):
        g = self._host(gate).reshape(-1)
        if g.size != want:
            raise PanicException("Incorrect len of the gate's buffer.")
        return g

    def _pos1(self, pos):
        if pos >= self.qubits_number:
            raise PanicException("pos is out of the bound.")

    def _pos2(self, pos2, pos1):
        if pos1 == pos2:
            raise PanicException("pos1 and pos2 must be different.")
        if pos1 >= self.qubits_number:
            raise PanicException("pos1 is out of the bound.")
        if pos2 >= self.qubits_number:
            raise PanicException("pos2 is out of the bound.")

    def apply_q1_gate(self, gate, pos):
        g = self._gate(gate, 4)
        self._pos1(pos)
        check(self._lib.q1gate(self._p, ptr(g), pos, self.qubits_number))

    def apply_q1_gate_inv(self, gate, pos):
        g = self._gate(gate, 4)
        self._pos1(pos)
        check(self._lib.q1gate_inv(self._p, ptr(g), pos, self.qubits_number))

    def apply_q1_gate_tr(self, gate, pos):
        self.apply_q1_gate(self._host(gate).reshape(2, 2).T.reshape(-1), pos)

    def apply_q1_gate_conj_tr(self, gate, pos):
        self.apply_q1_gate(self._host(gate).reshape(2, 2).T.conj().reshape(-1), pos)

    def apply_q2_gate(self, gate, pos2, pos1):
        g = self._gate(gate, 16)
        self._pos2(pos2, pos1)
        check(self._lib.q2gate(self._p, ptr(g), pos2, pos1, self.qubits_number))

    def apply_qk_gate(self, gate, positions):
        """Dense k-qubit gate, 1 <= k <= 5 (include/qdc/dense.h; beyond the reference, whose
        gates stop at 2 qubits): gate is 2^k x 2^k row-major, local index bit (k-1-b) is
        qubit positions[b] (positions[0] most significant, as apply_q2_gate's pos2)."""
        pos = [int(p) for p in positions]
        k = len(pos)
        if not 1 <= k <= 5:
            raise PanicException("k must be in 1..5.")
        g = self._gate(gate, 1 << (2 * k))
        if len(set(pos)) != k:
            raise PanicException("positions must be different.")
        if max(pos) >= self.qubits_number:
            raise PanicException("pos is out of the bound.")
        arr = (C.c_size_t * k)(*pos)
        check(self._lib.qdc_qkgate(self._p, ptr(g), arr, k, self.qubits_number))

    def apply_q2_gate_inv(self, gate, pos2, pos1):
        g = self._gate(gate, 16)
        self._pos2(pos2, pos1)
        check(self._lib.q2gate_inv(self._p, ptr(g), pos2, pos1, self.qubits_number))

    def apply_q2_gate_tr(self, gate, pos2, pos1):
        self.apply_q2_gate(self._host(gate).reshape(4, 4).T.reshape(-1), pos2, pos1)

    def apply_q2_gate_conj_tr(self, gate, pos2, pos1):
        self.apply_q2_gate(self._host(gate).reshape(4, 4).T.conj().reshape(-1), pos2, pos1)

    def apply_q2_gate_diag(self, gate, pos2, pos1):
        g = self._gate(gate, 4)
        self._pos2(pos2, pos1)
        check(self._lib.q2gate_diag(self._p, ptr(g), pos2, pos1, self.qubits_number))

    def apply_q2_gate_diag_conj(self, gate, pos2, pos1):
        self.apply_q2_gate_diag(self._host(gate).conj(), pos2, pos1)

    def get_q1_density(self, pos) -> np.ndarray:
        d = np.zeros(4, self.dtype)
        check(self._lib.get_q1density(self._p, ptr(d), pos, self.qubits_number))
        return d

    def get_q2_density(self, pos2, pos1) -> np.ndarray:
        d = np.zeros(16, self.dtype)
        check(self._lib.get_q2density(self._p, ptr(d), pos2, pos1, self.qubits_number))
        return d


def data_transfer(src: QuantizedTensor, dst: QuantizedTensor):
    """quantized_tensor.rs:169-176."""
    if src.qubits_number != dst.qubits_number:
        raise PanicException("fwd and bwd have different lengths.")
    src._lib.copy(src._p, dst._p, src.qubits_number)


def _grad(fn, fwd, bwd, width, *pos):
    if fwd.qubits_number != bwd.qubits_number:
        raise PanicException("fwd and bwd have different lengths.")
    g = np.zeros(width, fwd.dtype)
    check(getattr(fwd._lib, fn)(fwd._p, bwd._p, ptr(g), *pos, fwd.qubits_number))
    return g


def get_q1_grad(fwd, bwd, pos):
    """quantized_tensor.rs:178-189 (here the C error is checked; the reference ignores it)."""
    return _grad("q1grad", fwd, bwd, 4, pos)


def get_q2_grad(fwd, bwd, pos2, pos1):
    """quantized_tensor.rs:191-205."""
    return _grad("q2grad", fwd, bwd, 16, pos2, pos1)


def get_q2_grad_diag(fwd, bwd, pos2, pos1):
    """quantized_tensor.rs:207-221."""
    return _grad("q2grad_diag", fwd, bwd, 4, pos2, pos1)
