"""Save the GPU outputs of one fused v2 decode case (configs[4] seed) for offline comparison."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "ssnt-tts-rust_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import oracle as O  # noqa: E402
import ssnt_tts_amd as S  # noqa: E402
import test_gpu_fused_decode as t  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
lg, il, ol, d = t._config5(O, seed)
D = 16
g = S.v2_lattice_beam_search_decode(t._t(lg), t._t(np.arange(D, dtype=np.int32)), t._t(il),
                                    t._t(ol), 4, 0, False, False)
np.savez(ROOT / "gpurun_out" / f"fused_dbg_{seed}.npz", **{k: v.cpu().numpy() for k, v in g.items()})
print("saved")
