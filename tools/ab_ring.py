"""A/B of the fwd-bwd ring size (tuning; diagnostic only)."""
import json
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent))
from ab_fwd_bwd import bench_shape  # noqa: E402
for T in (100, 120):
    print(f"T{T}", json.dumps(bench_shape(256, T, 80, variants=(0, 8), rounds=5)), flush=True)
print("T200", json.dumps(bench_shape(256, 200, 80, variants=(0,), rounds=5)), flush=True)
