"""One dense k-qubit sample (bench.dense_gate_sample: k = 3, 4, 5, 8 gates each, n = 28 f32)
for rocprofv3 kernel traces and counter passes; prints its JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

print(json.dumps(bench.dense_gate_sample(argparse.Namespace(precision="f32"), 28)), flush=True)
