#!/usr/bin/env python3
"""Config C3 (VQSE, n = 26 f64) loss-and-gradient calls as bench.py's vqse_sample runs them,
once, for rocprofv3 kernel traces and PMC passes of the f64 path (profiles/r2*_f64_*)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

r = bench.vqse_sample()
print(json.dumps({k: r[k] for k in ("s_per_loss_grad_call", "energy", "device_ms_per_call", "host_ms_per_call")}),
      json.dumps(r.get("roofline")), flush=True)
