#!/usr/bin/env python3
"""Dense k-qubit MFMA kernels (k_qk): batches per wave iteration doubled or not
(QDC_QK_WIDE=1/0; QDC_QK_PAIR=0/1 for the paired-group 16-B accesses with --pair;
QDC_QK_PF=1/0 software-pipelined batches with --pf), n = 28 f32,
bench.py's dense_gate_sample (timing probe)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

args = argparse.Namespace(precision="f32")
knob = "QDC_QK_PAIR" if "--pair" in sys.argv else "QDC_QK_PF" if "--pf" in sys.argv else "QDC_QK_WIDE"
for rep in range(2):
    for v in ("1", "0"):
        os.environ[knob] = v
        print(knob, v, json.dumps(bench.dense_gate_sample(args, 28)), flush=True)
