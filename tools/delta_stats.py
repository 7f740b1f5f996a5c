"""Per-window partial-summary (delta) sizes of the headline stream on one rank, and the share of
pairs whose root is the giant's root (what a 4-byte 'joins the giant' encoding would save).
usage (GPU box): python tools/delta_stats.py [windows] [window_log2]"""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu
from gsgpu import gen

scale = 26; V = 1 << scale
nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 24)
s = torch.empty(nwin * W, dtype=torch.int32, device="cuda"); d = torch.empty(nwin * W, dtype=torch.int32, device="cuda")
for w in range(nwin):
    gen.rmat(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W], w * W, scale, 1)
ds = gsgpu.DisjointSet(V, id_bits=32, track_marks=True, stream=torch.cuda.current_stream())
out = torch.empty(4 * V, dtype=torch.int32, device="cuda")
tot_pairs = tot_giant = 0
for w in range(nwin):
    ds.fold(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W])
    n = ds.export_marks(out)
    pairs = out[:2 * n].view(n, 2)
    if n:
        roots = pairs[:, 1]
        vals, cnts = torch.unique(roots, return_counts=True)
        g = int(cnts.max())
    else:
        g = 0
    tot_pairs += n; tot_giant += g
    ds.close_window()
    print("window %3d pairs %9d giant-root pairs %9d (%.3f)" % (w + 1, n, g, g / max(n, 1)), flush=True)
print("summary: pairs %d, giant-root share %.3f, bytes as pairs %.1f MB, with 4-B giant joins %.1f MB" %
      (tot_pairs, tot_giant / max(tot_pairs, 1), 8e-6 * tot_pairs, 1e-6 * (8 * (tot_pairs - tot_giant) + 4 * tot_giant)))
