import sys
sys.path.insert(0, ".")
import bench
args = bench.parse([])
for rep in range(2):
    print(bench.dense_gate_sample(args, 28), flush=True)
