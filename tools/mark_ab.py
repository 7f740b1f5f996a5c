"""A/B of the steady fold with and without the hook log (GS_CC_TRACK_MARKS: what every multi-GPU
rank keeps for its partial-summary exports): RMAT-26, windows of 2^W edges, fold + close per window,
k_fold_ring time by HIP events. usage (GPU box): python tools/mark_ab.py [window_log2] [windows]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu  # noqa: E402
from gsgpu import gen  # noqa: E402
from gsgpu._abi import GS_K_RING, GS_K_COMPRESS, GS_TIMING_MASK  # noqa: E402

wl = int(sys.argv[1]) if len(sys.argv) > 1 else 21
nwin = int(sys.argv[2]) if len(sys.argv) > 2 else 256
scale, W = 26, 1 << wl
s = torch.empty(nwin * W, dtype=torch.int32, device="cuda")
d = torch.empty(nwin * W, dtype=torch.int32, device="cuda")
gen.rmat(s, d, 0, scale, 1)
torch.cuda.synchronize()
out = {"window_edges": W, "windows": nwin}
for marks in (False, True, False, True):
    ds = gsgpu.DisjointSet(1 << scale, id_bits=32, track_marks=marks, stream=torch.cuda.current_stream())
    ds.fold_windows(s, d, W)                                   # warm-up pass
    ds.reset()
    ds.timing(GS_TIMING_MASK | (1 << GS_K_RING) | (1 << GS_K_COMPRESS))
    ds.fold_windows(s, d, W)
    torch.cuda.synchronize()
    ms, n = ds.kernel_time(GS_K_RING)
    cms, cn = ds.kernel_time(GS_K_COMPRESS)
    key = "marks" if marks else "plain"
    out.setdefault(key, []).append({"ring_us_per_launch": 1e3 * ms / max(n, 1), "launches": n,
                                    "close_us": 1e3 * cms / max(cn, 1)})
    ds.close()
print(json.dumps(out))
