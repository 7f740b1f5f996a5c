import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import gsgpu
from pyoracle import coracle, EMIT_DENSE
o = coracle()
cap = 1 << 17; n = 100003
s, d = o.gen_er(0, n, cap, 5)
want = o.run(s, d, 0, emit=EMIT_DENSE, label_cap=cap)["labels"][0]
ts = torch.from_numpy(s.astype(np.int32)).cuda(); td = torch.from_numpy(d.astype(np.int32)).cuda()
def check(name, ds):
    lab = ds.dense().astype(np.int64)
    bad = np.nonzero(lab != want)[0]
    print(name, "mismatches", bad.size, "seen gpu", (lab >= 0).sum(), "seen want", (want >= 0).sum(), flush=True)
    if bad.size:
        print("  first:", [(int(v), int(lab[v]), int(want[v])) for v in bad[:10]])
        par = torch.empty(cap, dtype=torch.int32, device="cuda")
    return bad.size
a = gsgpu.DisjointSet(cap, id_bits=32); a.fold(ts, td); a.close_window(); check("parallel-full", a)
for chunk in (4, 64, 1024, 20000):
    b = gsgpu.DisjointSet(cap, id_bits=32)
    for lo in range(0, n, chunk):
        b.fold(ts[lo:lo+chunk], td[lo:lo+chunk])
    b.close_window(); check("chunk%d" % chunk, b)
# host-pointer path
c = gsgpu.DisjointSet(cap, id_bits=32); c.fold(s.astype(np.int32), d.astype(np.int32)); c.close_window(); check("host", c)
c = gsgpu.DisjointSet(cap, id_bits=64); c.fold(s, d); c.close_window(); check("host64", c)
# without close_window: find-based labels
e = gsgpu.DisjointSet(cap, id_bits=32); e.fold(ts, td)
r = e.find_batch(np.arange(cap)); bad = np.nonzero(r != want)[0]; print("find-based mismatches", bad.size, [(int(v), int(r[v]), int(want[v])) for v in bad[:10]])
# RMAT same size
s2, d2 = o.gen_rmat(0, n, 17, 5)
want = o.run(s2, d2, 0, emit=EMIT_DENSE, label_cap=cap)["labels"][0]
f = gsgpu.DisjointSet(cap, id_bits=32); f.fold(s2.astype(np.int32), d2.astype(np.int32)); f.close_window(); check("rmat17", f)
