import sys, json; sys.path.insert(0, "tools")
import bench_configs as bc
bc.cpu_time = lambda fn, min_s=0: 1.0
print(json.dumps(bc.v2_fwd_bwd_config(64, 400, 2000, 16, iters=2)))
