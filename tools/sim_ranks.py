"""Multi-rank CombineCC on ONE GPU: P device summaries stand in for P ranks (what bench.py runs
one per GPU), the exchange is replayed with device buffers handed across directly, and every
step is timed with HIP events. Measures what a multi-GPU run cannot show from a 1-GPU box: the
payload (pairs) each exchange moves per window and the merge folds on the receiving ranks; the
xGMI transfer time is modelled as bytes / 150 GB/s per link.

usage (GPU box): python tools/sim_ranks.py P windows [scheme ...]   schemes: gather tree allgather
(allgather: every rank keeps the global summary; per window each rank's delta goes to every other
rank over its own link and every rank folds the others' deltas with marking paused)
"""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "tests")]
import gsgpu
from gsgpu import gen
from gloo_tree import fold_slots, tree_schedule
from gsgpu._abi import GS_K_FOLD, GS_K_COMPRESS

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
NW = int(sys.argv[2]) if len(sys.argv) > 2 else 16
schemes = sys.argv[3:] or ["gather", "tree"]
scale = int(os.environ.get("SIM_SCALE", "26")); V = 1 << scale
W = 1 << int(os.environ.get("SIM_WLOG2", "24"))
LINK = 150e9

s = torch.empty(W, dtype=torch.int32, device="cuda"); d = torch.empty(W, dtype=torch.int32, device="cuda")
buf = torch.empty(2 * V, dtype=torch.int32, device="cuda")
ev = lambda: torch.cuda.Event(enable_timing=True)


def timed(fn):
    a, b = ev(), ev()
    a.record(); r = fn(); b.record(); b.synchronize()
    return r, a.elapsed_time(b) * 1e3          # us


# warm every kernel variant once (code-object loads stay out of the timings)
_wa = gsgpu.DisjointSet(V, id_bits=32, track_marks=True, stream=torch.cuda.current_stream())
_wb = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
for _w in range(3):
    gen.rmat(s, d, _w * W, scale, 1)
    _wa.fold(s, d); _wb.fold(s, d)
    _wb.fold_pairs(buf, _wa.export_marks(buf), id_bits=32)
    _wa.close_window(); _wb.close_window()
_wa.close(); _wb.close()
torch.cuda.synchronize()

for scheme in schemes:
    ag = scheme == "allgather"       # replicated summaries: every rank folds every other rank's delta
    ranks = [gsgpu.DisjointSet(V, id_bits=32, track_marks=(ag or r != 0), stream=torch.cuda.current_stream()) for r in range(P)]
    if ag:
        dbufs = [torch.empty(4 * V, dtype=torch.int32, device="cuda") for _ in range(P)]   # 2V pairs: the export contract
        rbuf = [torch.empty(2, dtype=torch.int32, device="cuda")]
    scheds = [tree_schedule(r, P) for r in range(P)]
    print("== %s P=%d scale=%d W/rank=2^%d" % (scheme, P, scale, W.bit_length() - 1), flush=True)
    tot = dict(fold=0.0, close=0.0, crit=0.0, xfer=0.0, merge=0.0, pairs=0)
    for w in range(NW):
        fold_us = []
        for r in range(P):
            gen.rmat(s, d, w * W * P + r * W, scale, 1)
            _, t = timed(lambda: ranks[r].fold(s, d))
            fold_us.append(t)
        merge_us, xfer_us, npairs = 0.0, 0.0, []
        if ag:
            tex = []
            cnt_dev = torch.zeros(P, dtype=torch.int64, device="cuda")
            for r in range(P):
                _, te = timed(lambda: ranks[r].export_marks_async(dbufs[r], cnt_dev[r:r + 1]))
                tex.append(te)
            ns = [int(x) for x in cnt_dev.tolist()]
            if os.environ.get("SIM_VERBOSE") and w in (0, 15, 63):
                print("   w%d export wall us %s" % (w + 1, ["%.0f" % x for x in tex]), flush=True)
            npairs = ns
            m = max(ns)
            xfer_us = max(tex) + 8 * m / LINK * 1e6           # all pairs of links at once
            # AllgatherMerge's layout: P slots of m pairs, each padded with copies of its first pair
            for q in range(P):
                if 0 < ns[q] < m:
                    dbufs[q][2 * ns[q]: 2 * m].view(-1, 2).copy_(dbufs[q][0:2].view(1, 2).expand(m - ns[q], 2))
            if m:
                if rbuf[0].numel() < 2 * P * m:
                    rbuf[0] = torch.empty(2 * P * m, dtype=torch.int32, device="cuda")
                torch.cat([dbufs[q][:2 * m] for q in range(P)], out=rbuf[0][:2 * P * m])
            mt = []
            for r in range(P):
                ranks[r].set_marking(False)
                _, tf = timed(lambda: fold_slots(ranks[r], rbuf[0], m, [0 if q == r else ns[q] for q in range(P)]) if m else None)
                ranks[r].set_marking(True)
                mt.append(tf)
            merge_us = max(mt)
            if os.environ.get("SIM_VERBOSE") and w < 3:
                print("   w%d deltas %s merge %s" % (w + 1, ns, ["%.0f" % x for x in mt]), flush=True)
        elif scheme == "gather":
            per = []
            for r in range(1, P):
                n, te = timed(lambda: ranks[r].export_marks(buf))
                _, tf = timed(lambda: ranks[0].fold_pairs(buf, n, id_bits=32))
                npairs.append(n); merge_us += tf; per.append(te + 8 * n / LINK * 1e6)
                if os.environ.get("SIM_VERBOSE") and w < 2:
                    print("   w%d rank %d: %d pairs, export %.0f us, merge fold %.0f us" % (w + 1, r, n, te, tf), flush=True)
            xfer_us = max(per) if per else 0.0            # every peer over its own link, at once
        else:                                            # tree: rounds in sequence
            for i in range(len(scheds[0])):
                rnd_x, rnd_m = 0.0, 0.0
                for r in range(P):
                    role, peer = scheds[r][i]
                    if role == "send":
                        n, te = timed(lambda: ranks[r].export_marks(buf))
                        _, tf = timed(lambda: ranks[peer].fold_pairs(buf, n, id_bits=32))
                        npairs.append(n)
                        rnd_x = max(rnd_x, te + 8 * n / LINK * 1e6)
                        rnd_m = max(rnd_m, tf)
                xfer_us += rnd_x; merge_us += rnd_m
        close_us = []
        for r in range(P):
            _, t = timed(lambda: ranks[r].close_window())
            close_us.append(t)
        crit = max(fold_us) + xfer_us + merge_us + (max(close_us) if ag else close_us[0])
        tot["fold"] += max(fold_us); tot["close"] += close_us[0]; tot["crit"] += crit
        tot["xfer"] += xfer_us; tot["merge"] += merge_us; tot["pairs"] += sum(npairs)
        print("w%3d fold max %6.0f us (r0 %6.0f)  pairs %8d (max %7d)  xfer %6.0f  merge folds %6.0f  close r0 %5.0f  "
              "critical %6.0f us" % (w + 1, max(fold_us), fold_us[0], sum(npairs), max(npairs or [0]), xfer_us,
                                     merge_us, close_us[0], crit), flush=True)
    print("TOTAL %s: fold %.2f ms, xfer %.2f, merge %.2f, close %.2f, critical %.2f ms -> efficiency vs no-merge %.3f, "
          "pairs %d" % (scheme, tot["fold"] / 1e3, tot["xfer"] / 1e3, tot["merge"] / 1e3, tot["close"] / 1e3,
                        tot["crit"] / 1e3, (tot["fold"] + tot["close"]) / tot["crit"], tot["pairs"]), flush=True)
    for r in ranks:
        r.close()
    torch.cuda.synchronize()
