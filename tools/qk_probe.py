#!/usr/bin/env python3
"""Dense k-qubit MFMA kernels (k_qk) with and without the paired-group 16-B accesses
(QDC_QK_PAIR=0/1), n = 28 f32, bench.py's dense_gate_sample (timing probe)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

args = argparse.Namespace(precision="f32")
for rep in range(2):
    for pair in ("1", "0"):
        os.environ["QDC_QK_PAIR"] = pair
        print("pair", pair, json.dumps(bench.dense_gate_sample(args, 28)), flush=True)
