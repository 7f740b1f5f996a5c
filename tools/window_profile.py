"""Per-window fold profile of the headline stream (RMAT-26, 2^24-edge windows): fold time per
window (HIP events) and, with GSGPU_FOLD_STATS=1, the fold's path counters per window.
usage (GPU box): python tools/window_profile.py [windows]"""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu
from gsgpu import gen
from gsgpu._abi import GS_K_FOLD, GS_K_COMPRESS

scale = 26; V = 1 << scale; W = 1 << 24
nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 64
s = torch.empty(nwin * W, dtype=torch.int32, device="cuda"); d = torch.empty(nwin * W, dtype=torch.int32, device="cuda")
for w in range(nwin):
    gen.rmat(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W], w * W, scale, 1)
torch.cuda.synchronize()
ds = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
for rep in range(2):
    ds.reset()
    ds.timing(True)
    prev_f = prev_c = 0.0
    rows = []
    for w in range(nwin):
        ds.fold(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W])
        ds.close_window()
        f, _ = ds.fold_time(); c, _ = ds.kernel_time(GS_K_COMPRESS)
        rows.append((w + 1, (f - prev_f) * 1e3, (c - prev_c) * 1e3))
        prev_f, prev_c = f, c
    ds.timing(False)
for r in rows:
    print("window %3d  fold %8.1f us  close %6.1f us" % r, file=sys.stderr if False else sys.stdout, flush=True)
young = [r for r in rows if r[0] <= 12]
steady = [r for r in rows if r[0] > 12]
print("summary: fold w1 %.1f us, w2-12 %.1f us, steady mean %.1f us (%d windows), close total %.1f us, step fold+close %.1f us"
      % (rows[0][1], sum(r[1] for r in young[1:]), sum(r[1] for r in steady) / max(len(steady), 1), len(steady),
         sum(r[2] for r in rows), sum(r[1] + r[2] for r in rows)), flush=True)
