"""GPU EXACT-mode replicas (bench.gpu_exact_replicas): aggregate nodes/s of R independent EXACT planner processes on
one GPU, for R in argv (default 1 2 4 8 16); cfg3 scene, 2 s queries."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[1:] if "=" in kv}  # engine options, k=v
    for R in [int(x) for x in sys.argv[1:] if "=" not in x] or [1, 2, 4, 8, 16]:
        r = bench.gpu_exact_replicas("cfg3", 2000.0, R, 1, opts=opts)
        print(f"R {R:2d} {opts}: {r['value']:8.0f} nodes/s aggregate ({r['value'] / R:7.0f} per replica); {r['sample']}",
              flush=True)
