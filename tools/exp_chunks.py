import sys, os, time, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu
from gsgpu import gen
scale = 26; V = 1 << scale; W = 1 << 24; NW = 8
s = torch.empty(NW * W, dtype=torch.int32, device="cuda"); d = torch.empty(NW * W, dtype=torch.int32, device="cuda")
gen.rmat(s, d, 0, scale, 1); torch.cuda.synchronize()
ds = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
def fold_chunked(lo, hi, chunk, close_after=None):
    a = lo
    while a < hi:
        b = min(hi, a + chunk(a - lo))
        ds.fold(s[a:b], d[a:b]); a = b
        if close_after is not None and (a - lo) in close_after: ds.close_window()
def run(name, chunk, close_after=None, reps=2):
    res = []
    for _ in range(reps):
        ds.reset(); torch.cuda.synchronize()
        times = []
        for w in range(NW):
            t0 = time.perf_counter()
            fold_chunked(w * W, (w + 1) * W, chunk, close_after if w == 0 else None)
            ds.close_window(); torch.cuda.synchronize(); times.append((time.perf_counter() - t0) * 1e3)
        res.append(times)
    r = np.min(np.array(res), axis=0)
    print("%-28s w1 %.2f  w2 %.2f  w3 %.2f  w8 %.2f  total %.2f" % (name, r[0], r[1], r[2], r[7], r.sum()), flush=True)
run("whole windows", lambda off: W)
for c in (1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 22):
    run("chunk %dK" % (c >> 10), lambda off, c=c: c)
run("geometric 64K->", lambda off: max(1 << 16, min(W, off)))
run("geometric 256K->", lambda off: max(1 << 18, min(W, off)))
run("geometric 256K-> 4M cap", lambda off: max(1 << 18, min(1 << 22, off)))
run("256K + close@1M", lambda off: 1 << 18, close_after={1 << 20})
run("256K + close@1M,4M", lambda off: 1 << 18, close_after={1 << 20, 1 << 22})
