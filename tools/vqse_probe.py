#!/usr/bin/env python3
"""Config C3 (VQSE, n = 26 f64) seconds per loss-and-gradient call with the f64 gate passes
register-resident (QDC_RQ64=1, k_rw) or in LDS tiles (QDC_RQ64=0, k_fused); bench.py's
vqse_sample (timing probe)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

for rep in range(2):
    for v in ("1", "0"):
        os.environ["QDC_RQ64"] = v
        r = bench.vqse_sample()
        print("rq64", v, json.dumps({k: r[k] for k in ("s_per_loss_grad_call", "energy", "device_ms_per_call")}),
              json.dumps(r.get("kernels")), flush=True)
