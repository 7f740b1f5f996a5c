import sys, os, time, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu
from gsgpu import gen
scale = 26; V = 1 << scale; W = 1 << 24
s = torch.empty(4 * W, dtype=torch.int32, device="cuda"); d = torch.empty(4 * W, dtype=torch.int32, device="cuda")
gen.rmat(s, d, 0, scale, 1); torch.cuda.synchronize()
ds = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
def t(fn, reps=3):
    out = []
    for _ in range(reps):
        ds.reset(); torch.cuda.synchronize(); t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); out.append((time.perf_counter() - t0) * 1e3)
    return " ".join("%.2f" % x for x in out)
def plan(cuts, close):
    def f():
        lo = 0
        for c in cuts + [W]:
            ds.fold(s[lo:c], d[lo:c]); lo = c
            if close and c != W: ds.close_window()
    return f
print("full window      ", t(plan([], False)), flush=True)
for k in (4, 16, 64):
    print("chunks %-3d       " % k, t(plan([W * i // k for i in range(1, k)], False)), flush=True)
for cuts in ([1 << 20], [1 << 18, 1 << 20], [1 << 16, 1 << 18, 1 << 20, 1 << 22], [1 << 20, 1 << 22], [1 << 22]):
    print("compress at %-30s" % [c >> 10 for c in cuts], t(plan(cuts, True)), flush=True)
# steady state for reference: windows 2..4 after window 1
def steady():
    for w in range(1, 4):
        ds.fold(s[w*W:(w+1)*W], d[w*W:(w+1)*W]); ds.close_window()
ds.reset(); ds.fold(s[:W], d[:W]); ds.close_window(); torch.cuda.synchronize()
t0 = time.perf_counter(); steady(); torch.cuda.synchronize(); print("windows 2-4 ms", (time.perf_counter() - t0) * 1e3)
