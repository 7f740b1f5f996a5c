"""The real GS_MERGE_PREFILTER protocol (broadcast schedule, stale bitmaps, senders' own hot / warm
sets) over the in-process transport on one GPU, strong layout of BASELINE config 3 (RMAT-26, 64
global windows of 2^24 edges, bench.py's default rank-0 share): run with GSGPU_PREFILTER_LOG=1, the
senders' survivor counts go to stderr; this prints their total next to what tools/sim_ranks.py's
filter against the Merger's current state let through (a lower bound).
usage (GPU box): GSGPU_PREFILTER_LOG=1 python tools/prefilter_survivors.py P 2> log; grep survivors log"""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gelly-streaming_amd")]

import torch  # noqa: E402
import gsgpu  # noqa: E402
from gsgpu import Comm, gen  # noqa: E402
from bench import prefilter_share0  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N, W, scale = 64, 1 << 24, 26
V = 1 << scale
src = torch.empty(N * W, dtype=torch.int32, device="cuda")
dst = torch.empty(N * W, dtype=torch.int32, device="cuda")
for w in range(N):
    gen.rmat(src[w * W:(w + 1) * W], dst[w * W:(w + 1) * W], w * W, scale, 1)
torch.cuda.synchronize()
W1 = int(W * (1 - prefilter_share0(P)) / (P - 1)) // 4 * 4
if W - (P - 1) * W1 < 4:
    W1 -= 4
W0 = W - (P - 1) * W1
sl = [(0, W0)] + [(W0 + (q - 1) * W1, W1) for q in range(1, P)]
comms = Comm.local_group(P, 0)
errors = []


merge_ms = [0.0, 0]


def rank(r):
    try:
        ds = gsgpu.DisjointSet(V, id_bits=32)
        if r == 0:                                   # the Merger's survivor folds (GS_K_MERGE launches)
            from gsgpu._abi import GS_K_MERGE, GS_TIMING_MASK
            ds.timing(GS_TIMING_MASK | (1 << GS_K_MERGE))
        off, ln = sl[r]
        for w in range(N):
            lo = w * W + off
            ds.fold_windows(src[lo:lo + ln], dst[lo:lo + ln], ln, comm=comms[r], mode="prefilter")
        if r == 0:
            from gsgpu._abi import GS_K_MERGE
            merge_ms[0], merge_ms[1] = ds.kernel_time(GS_K_MERGE)
        ds.close()
    except Exception as e:                                       # noqa: BLE001
        errors.append((r, repr(e)))


th = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
for t in th:
    t.start()
for t in th:
    t.join(timeout=900)
for c in comms:
    c.close()
print({"P": P, "rank0_edges": W0, "sender_edges": W1, "errors": errors,
       "rank0_merge_ms": round(merge_ms[0], 3), "rank0_merge_launches": merge_ms[1]}, flush=True)
