"""A/B of the fwd-bwd kernels at the long-form shape (configs[4]; diagnostic only)."""
import json
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent))
from ab_fwd_bwd import bench_shape  # noqa: E402
print("64x2000x400", json.dumps(bench_shape(64, 2000, 400, variants=(0, 1), rounds=3, iters=3)), flush=True)
print("64x400x400", json.dumps(bench_shape(64, 400, 400, variants=(0, 1), rounds=3, iters=5)), flush=True)
print("256x200x200", json.dumps(bench_shape(256, 200, 200, variants=(0, 1), rounds=3, iters=5)), flush=True)
