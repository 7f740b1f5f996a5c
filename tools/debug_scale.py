import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")]
import gsgpu
from gsgpu import gen
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
V, E, W = 1 << scale, 16 << scale, 1 << scale
s = torch.empty(E, dtype=torch.int32, device="cuda"); d = torch.empty(E, dtype=torch.int32, device="cuda")
gen.rmat(s, d, 0, scale, 1); torch.cuda.synchronize()
sl, dl = s.long(), d.long()
def bad_edges(lab):
    return int((lab[sl] != lab[dl]).sum())
def run(name, windows, close_each, use_find):
    ds = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
    for lo in range(0, E, windows):
        ds.fold(s[lo:lo+windows], d[lo:lo+windows])
        if close_each: ds.close_window()
    if use_find:
        ids = torch.arange(V, dtype=torch.int32, device="cuda")
        r = torch.from_numpy(ds.find_batch(ids.cpu().numpy())).cuda()
        lab = r.long()
    else:
        lab = torch.empty(V, dtype=torch.int32, device="cuda"); ds.dense(out=lab); lab = lab.long()
    nb = bad_edges(lab)
    print(name, "bad edges", nb, "seen", int((lab >= 0).sum()), "labels>v", int((lab > torch.arange(V, device='cuda')).sum()), flush=True)
    return ds, lab
run("W=4M close-each dense", W, True, False)
run("W=4M no-close find", W, False, True)
run("W=4M no-close dense(compress once)", W, False, False)
run("single-window dense", E, False, False)
run("W=64K close-each dense", 1 << 16, True, False)
