#!/usr/bin/env python3
"""Dense k-qubit gates (k_qk) at n = 28 f32 by target placement (timing probe): the C = 2^k
amplitudes of a group sit C far-apart addresses when the targets are high qubits and within a
few KiB when they are low, so this separates the kernel's own rate from the cost of touching C
distant pages / DRAM rows at once.  Same per-kernel HIP-event timing as bench.dense_gate_sample."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
import quantum_differentiable_circuit as q  # noqa: E402

n = 28
rng = np.random.default_rng(2)
t = q.QuantizedTensor.new_standard(n, precision="f32")
places = {
    "low": lambda k: list(range(1, k + 1)),
    "mid": lambda k: list(range(10, 10 + k)),
    "high": lambda k: list(range(n - k, n)),
    "spread": lambda k: [int(round(1 + i * (n - 2) / (k - 1))) for i in range(k)],
}
for k in (3, 4, 5):
    u = np.ascontiguousarray(bench.O_haar(rng, 1 << k), dtype=np.complex64)
    for name, f in places.items():
        pos = f(k)
        t.apply_qk_gate(u, pos)  # warm-up
        q.primitives_sync("f32")
        q.primitives_profile(True, "f32")
        for _ in range(6):
            t.apply_qk_gate(u, pos)
        s = q.primitives_profile_collect("f32")[f"qk{k}"]
        q.primitives_profile(False, "f32")
        gbs = s["algo_bytes"] / (s["total_ms"] * 1e-3) / 1e9
        print(json.dumps({"k": k, "place": name, "pos": pos, "GB/s": round(gbs, 1),
                          "frac": round(gbs / bench.HBM_PEAK_GBS, 4),
                          "avg_ms": round(s["total_ms"] / s["launches"], 4)}), flush=True)
args = type("A", (), {"precision": "f32"})()
print(json.dumps({"bench_dense_gate_sample": bench.dense_gate_sample(args, n)}), flush=True)
