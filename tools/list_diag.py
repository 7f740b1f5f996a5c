"""Diagnose a list-close parity failure: per window, GPU dense labels vs scipy connected components
(min-id label of every seen vertex). usage: python tools/list_diag.py [windows]"""
import os, sys
import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gelly-streaming_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
from gsgpu import DisjointSet
from pyoracle import coracle
from test_gpu_listclose import _fold_window

def want_labels(s, d, cap):
    g = sp.coo_matrix((np.ones(s.size), (s, d)), shape=(cap, cap))
    nc, lab = connected_components(g, directed=False)
    seen = np.zeros(cap, bool); seen[s] = True; seen[d] = True
    mn = np.full(nc, cap, np.int64)
    np.minimum.at(mn, lab, np.arange(cap))
    out = np.where(seen, mn[lab], -1)
    return out

o = coracle()
scale, n, W = 16, 1 << 19, 4096
cap = 1 << scale
s, d = o.gen_rmat(0, n, scale, 11)
ts = torch.from_numpy(s.astype(np.int32)).cuda(); td = torch.from_numpy(d.astype(np.int32)).cuda()
from pyoracle import EMIT_CHECKSUM
wantc = [int(x) for x in o.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap)["checksums"]]
ds = DisjointSet(cap, id_bits=32, stream=torch.cuda.current_stream())
nw = int(sys.argv[1]) if len(sys.argv) > 1 else 24
for w, lo in enumerate(range(0, n, W)):
    if w >= nw: break
    _fold_window(ds, torch, ts, td, lo, min(n, lo + W), w)
    ds.close_window()
    if w % 13 == 7:
        ds.close_window()
    h = ds.checksum()[0]
    got = ds.dense().astype(np.int64)
    print("window %d checksum %s want %s" % (w, h, wantc[w]), flush=True)
    want = want_labels(s[:lo + W], d[:lo + W], cap)
    bad = np.nonzero(got != want)[0]
    from pyoracle import dense_checksum
    print("  dense_checksum(got) %s dense_checksum(want) %s" % (dense_checksum(got)[0], dense_checksum(want)[0]))
    print("window %d: %d bad" % (w, bad.size), flush=True)
    if bad.size:
        for v in bad[:10]:
            print("  v=%d got=%d want=%d  parent(got)=%d want(got)=%d" % (v, got[v], want[v], got[got[v]] if got[v] >= 0 else -9, want[got[v]] if got[v] >= 0 else -9))
        break
