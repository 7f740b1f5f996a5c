"""Multi-rank CombineCC on ONE GPU: P device summaries stand in for P ranks (what bench.py runs
one per GPU), the exchange is replayed with device buffers handed across directly, and every
step is timed with HIP events. Measures what a multi-GPU run cannot show from a 1-GPU box: the
payload (pairs) each exchange moves per window and the merge folds on the receiving ranks; the
xGMI transfer time is modelled as bytes / 150 GB/s per link.

usage (GPU box): python tools/sim_ranks.py P windows [scheme ...]   schemes: gather tree allgather prefilter prefilter_r05 prefilter_forest
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

KT = not os.environ.get("SIM_WALL")     # kernel time (HIP events on the launches) + GAP per boundary;
GAP = 3.0                               # SIM_WALL=1: the round-1..4 wall accounting per operation


def op(h, fn):
    """(result, us) of fn's work on handle h: its kernels' time (KT) or the wall time of the op."""
    if not KT:
        return timed(fn)
    k0 = sum(h.kernel_time(k)[0] for k in range(6))
    r = fn()
    torch.cuda.synchronize()
    return r, (sum(h.kernel_time(k)[0] for k in range(6)) - k0) * 1e3


def one_gpu_base(P, NW):
    """The one-GPU reference on the same clock: whole global windows folded and closed."""
    one = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
    one.timing(True)
    wa = torch.empty(W * P, dtype=torch.int32, device="cuda")
    wb = torch.empty(W * P, dtype=torch.int32, device="cuda")
    base = 0.0
    for w in range(NW):
        gen.rmat(wa, wb, w * W * P, scale, 1)
        _, t1 = op(one, lambda: one.fold(wa, wb))
        _, t2 = op(one, lambda: one.close_window())
        base += t1 + t2 + (2 * GAP if KT else 0.0)
    one.close()
    print("one GPU, same stream: %.2f ms (%s)" % (base / 1e3, "kernel time + 2 launch gaps per window" if KT
                                                  else "wall time per operation"), flush=True)
    return base


def _bench_layout(P):
    """bench.py's per-rank slices of a global window under --merge prefilter (strong layout)."""
    import importlib
    sys.argv = sys.argv[:1]
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")

    class _L:
        edge_factor, scale, window_log2, scaling, share0, merge = 16, 26, 0, "strong", None, "prefilter"
    _L.scale = scale
    if os.environ.get("SIM_SHARE0"):                  # (bench.py --share0)
        _L.share0 = float(os.environ["SIM_SHARE0"])
    _L.window_log2 = (W * P).bit_length() - 1
    return [bench.layout(_L, P, r)[1] for r in range(P)]


# the round-6 broadcast schedule (csrc/comm.hip merge_prefilter): synchronous after the first
# kBcastSync closes, then asynchronous (installed by the senders kBcastLag windows later) after every
# close while w < 16, then after every 4th
SYNC, LAG = int(os.environ.get("SIM_SYNC", "1")), 2      # SIM_SYNC: another synchronous prefix (A/B)


def bcast_async(w):
    return w >= SYNC and (w < 16 or w % 4 == 3)


def sim_prefilter(P, NW, r05=False):
    """GS_MERGE_PREFILTER, the round-6 protocol (r05=True: round 5's accounting, kept for the record).
    The global window (P x the per-rank W) is split as bench.py splits it (rank 0 no slice at P = 8).
    Each sender slice is filtered against the Merger's giant state AS THE SENDER HAS IT — the state
    after the last close whose broadcast it has installed (a summary per sender replays the Merger's
    folds and closes that many windows behind, so the survivors include the stale bitmap's extra
    edges) — and rank 0 folds every survivor and closes. Per window: the senders' filters run while
    rank 0 folds and closes the previous window (the senders' send of window w waits for rank 0's
    receive, posted after its close of w - 1), so a window costs the longer of the two chains; a
    synchronous broadcast (after close 0; round 6's first protocol: 0 and 1) serialises them. Asynchronous broadcasts cost rank 0
    a snapshot copy (8 MiB) and the senders an install copy, on their chains."""
    s0 = max(0.0, 1.125 / P - 0.125)                                                   # bench.py prefilter_share0
    BCAST_BW = 64e9
    COPY_BW = 4.0e12                                  # D2D copy (read + write), snapshot / install
    base = one_gpu_base(P, NW)
    Wg = W * P
    if r05:
        share0 = float(os.environ.get("SIM_SHARE0", str(s0 if s0 >= 1.0 / 32 else 0.0)))
        W0 = max(4, int(Wg * share0) // 4 * 4)
        W1 = (Wg - W0) // (P - 1) // 4 * 4
        W0 = Wg - W1 * (P - 1)
        sizes = [W0] + [W1] * (P - 1)
    else:
        sizes = _bench_layout(P)
    W0 = sizes[0]
    m0 = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
    # one lagging summary per sender (SIM_SHARED_LAG=1: one for all, as the first round-6 model ran it):
    # each sender's hot set is admitted by its own filter launches (one per window, the protocol's
    # cadence); one handle running all P - 1 filters admitted P - 1 times as often
    nlag = 0 if r05 else (1 if os.environ.get("SIM_SHARED_LAG") else P - 1)
    lags = [gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream()) for _ in range(nlag)]
    lag = lags[0] if lags else None
    mx = max(sizes)
    ss = torch.empty(mx, dtype=torch.int32, device="cuda")
    sd = torch.empty(mx, dtype=torch.int32, device="cuda")
    outs = [torch.empty(2 * sizes[r], dtype=torch.int32, device="cuda") for r in range(1, P)]
    gbytes = V // 8
    m0.timing(True)
    for h in lags:
        h.timing(True)

    def ktime(h):
        return sum(h.kernel_time(k)[0] for k in range(6)) * 1e3        # us, cumulative

    def ktimed(h, fn):                                # (result, kernel-only us of the launches fn made)
        k0 = ktime(h)
        r = fn()
        torch.cuda.synchronize()
        return r, ktime(h) - k0
    print("== prefilter%s P=%d scale=%d global window 2^%d: rank 0 %d edges, senders %s each" %
          ("_r05" if r05 else "", P, scale, Wg.bit_length() - 1, W0, sorted(set(sizes[1:]))), flush=True)
    tot = dict(crit=0.0, filt=0.0, merge=0.0, close=0.0, own=0.0, surv=0)
    history = []                                      # per window: (own slice, all survivors) as folded by rank 0
    lag_at = -1                                       # lag summary = the Merger after close(lag_at)
    prev_r0 = 0.0                                     # rank 0's chain of the previous window (overlaps this filter)
    for w in range(NW):
        filt_h = m0
        if lag is not None:
            # the state the senders filter window w with: the last installed broadcast
            avail = [j for j in range(w) if (j < SYNC and j <= w - 1) or (bcast_async(j) and j + LAG <= w)]
            target = max(avail) if avail else -1
            while lag_at < target:
                lag_at += 1
                o, sv = history[lag_at]
                for h in lags:
                    if o is not None:
                        h.fold(o[0], o[1])
                    if sv is not None and sv.numel():
                        h.fold_pairs(sv, sv.numel() // 2, id_bits=32)
                    h.close_window()
            torch.cuda.synchronize()
            filt_h = lag
        own = None
        t0 = 0.0
        off = w * Wg
        if W0:
            gen.rmat(ss[:W0], sd[:W0], off, scale, 1)
            own = (ss[:W0].clone(), sd[:W0].clone())
            _, t0 = ktimed(m0, lambda: m0.fold(ss[:W0], sd[:W0]))
        off += W0
        ns, tf = [], []
        for r in range(1, P):
            n_r = sizes[r]
            gen.rmat(ss[:n_r], sd[:n_r], off, scale, 1)
            off += n_r
            fh = lags[(r - 1) % len(lags)] if lags else filt_h
            n, k = ktimed(fh, lambda: fh.filter_edges(ss[:n_r], sd[:n_r], outs[r - 1]))
            ns.append(n); tf.append(k)
        allp = torch.cat([outs[r - 1][:2 * ns[r - 1]] for r in range(1, P)])     # every survivor, one fold
        _, tm = ktimed(m0, lambda: m0.fold_pairs(allp, allp.numel() // 2, id_bits=32) if allp.numel() else None)
        _, tc = ktimed(m0, lambda: m0.close_window())
        if lag is not None:
            history.append((own, allp.clone()))
        xfer = max(8 * n / LINK * 1e6 for n in ns)
        if r05:
            due = w < 4 or w % 16 == 15
            bc = gbytes / BCAST_BW * 1e6 if due else 0.0
            crit = (max(max(tf) + xfer, t0) + tm + tc + bc) if due else max(max(tf) + xfer, t0 + tm + tc)
            crit += GAP * 4
        else:
            sync = w < SYNC
            bc = gbytes / BCAST_BW * 1e6 if sync else 0.0
            snap = 2 * gbytes / COPY_BW * 1e6 if bcast_async(w) else 0.0
            inst = 2 * gbytes / COPY_BW * 1e6 if (w >= LAG and bcast_async(w - LAG)) else 0.0
            chain_s = max(tf) + inst + xfer                            # senders: filter, send
            chain_r = (t0 + GAP if W0 else 0.0) + tm + tc + snap + 2 * GAP   # rank 0: (own,) fold, close
            if w == 0 or w - 1 < SYNC:
                # the filter of w waited for the broadcast after close(w - 1): nothing overlapped
                crit = chain_s + chain_r + bc
            else:
                crit = max(chain_s, chain_r) + bc
        tot["crit"] += crit; tot["filt"] += max(tf); tot["merge"] += tm; tot["close"] += tc; tot["own"] += t0
        tot["surv"] += sum(ns)
        print("w%3d own fold %6.0f us  sender filter max %6.0f us  survivors %8d (max %7d)  xfer %5.0f  "
              "merge folds %6.0f  close %5.0f  bcast %5.0f  critical %6.0f us" %
              (w + 1, t0, max(tf), sum(ns), max(ns), xfer, tm, tc, bc, crit), flush=True)
    print("TOTAL prefilter%s: own %.2f ms, sender filter %.2f, merge %.2f, close %.2f, critical %.2f ms, survivors %d; "
          "one GPU %.2f ms -> model speedup %.2fx at P=%d"
          % ("_r05" if r05 else "", tot["own"] / 1e3, tot["filt"] / 1e3, tot["merge"] / 1e3, tot["close"] / 1e3,
             tot["crit"] / 1e3, tot["surv"], base / 1e3, base / tot["crit"], P), flush=True)
    m0.close()
    for h in lags:
        h.close()
    torch.cuda.synchronize()


def sim_prefilter_forest(P, NW):
    """Round-6 prototype: GS_MERGE_PREFILTER whose senders keep a partition forest. Each sender
    filters its slice against the Merger's giant state (as sim_prefilter), folds the survivors into
    its OWN cumulative forest (UpdateCC per partition, hook log on) and sends the forest's delta —
    (v, root) pairs of the roots it hooked — instead of the raw survivors; the Merger folds the pairs
    (DisjointSet.merge) and closes. Same per-window accounting as sim_prefilter, with rank 0 folding
    no slice of its own (bench.py's layout at P = 8) and the sender chain = filter + forest fold +
    export."""
    BCAST_BW = 64e9
    base = one_gpu_base(P, NW)
    Wg = W * P
    W1 = Wg // (P - 1) // 4 * 4
    sizes = [W1] * (P - 1)
    for r in range((Wg - W1 * (P - 1)) // 4):
        sizes[r % (P - 1)] += 4
    m0 = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
    snd = [gsgpu.DisjointSet(V, id_bits=32, track_marks=True, stream=torch.cuda.current_stream()) for _ in range(P - 1)]
    mx = max(sizes)
    ss = torch.empty(mx, dtype=torch.int32, device="cuda")
    sd = torch.empty(mx, dtype=torch.int32, device="cuda")
    surv = torch.empty(2 * mx, dtype=torch.int32, device="cuda")
    pbuf = [torch.empty(4 * V, dtype=torch.int32, device="cuda") for _ in range(P - 1)]
    gbytes = V // 8
    for h in [m0] + snd:
        h.timing(True)

    def kt(h):
        return sum(h.kernel_time(k)[0] for k in range(6)) * 1e3

    def ktimed(h, fn):
        k0 = kt(h)
        r = fn()
        torch.cuda.synchronize()
        return r, kt(h) - k0
    print("== prefilter_forest P=%d scale=%d global window 2^%d: rank 0 no slice, senders %d edges each" %
          (P, scale, Wg.bit_length() - 1, mx), flush=True)
    tot = dict(crit=0.0, snd=0.0, merge=0.0, close=0.0, surv=0, pairs=0)
    for w in range(NW):
        chain, ns, npairs = [], [], []
        off = w * Wg
        for r in range(P - 1):
            n_r = sizes[r]
            gen.rmat(ss[:n_r], sd[:n_r], off, scale, 1)
            off += n_r
            n, tf = ktimed(m0, lambda: m0.filter_edges(ss[:n_r], sd[:n_r], surv))
            _, tl = ktimed(snd[r], lambda: snd[r].fold_pairs(surv, n, id_bits=32) if n else None)
            npr, te = ktimed(snd[r], lambda: snd[r].export_marks(pbuf[r]))
            chain.append(tf + tl + te + 2 * GAP)
            ns.append(n)
            npairs.append(npr)
        allp = torch.cat([pbuf[r][:2 * npairs[r]] for r in range(P - 1)])
        _, tm = ktimed(m0, lambda: m0.fold_pairs(allp, allp.numel() // 2, id_bits=32) if allp.numel() else None)
        _, tc = ktimed(m0, lambda: m0.close_window())
        xfer = max(8 * n / LINK * 1e6 for n in npairs)
        due = w < 4 or w % 16 == 15
        bc = gbytes / BCAST_BW * 1e6 if due else 0.0
        if due:
            crit = max(chain) + xfer + tm + tc + bc
        else:
            crit = max(max(chain) + xfer, tm + tc)
        crit += GAP * 3                               # rank 0's chain: receive, fold, close
        tot["crit"] += crit; tot["snd"] += max(chain); tot["merge"] += tm; tot["close"] += tc
        tot["surv"] += sum(ns); tot["pairs"] += sum(npairs)
        print("w%3d sender chain max %6.0f us  survivors %8d  pairs %8d (max %7d)  xfer %5.0f  merge folds %6.0f  "
              "close %5.0f  bcast %5.0f  critical %6.0f us" % (w + 1, max(chain), sum(ns), sum(npairs), max(npairs), xfer,
                                                               tm, tc, bc, crit), flush=True)
    print("TOTAL prefilter_forest: sender chain %.2f ms, merge %.2f, close %.2f, critical %.2f ms, survivors %d, pairs %d; "
          "one GPU %.2f ms -> model speedup %.2fx at P=%d"
          % (tot["snd"] / 1e3, tot["merge"] / 1e3, tot["close"] / 1e3, tot["crit"] / 1e3, tot["surv"], tot["pairs"],
             base / 1e3, base / tot["crit"], P), flush=True)
    for h in [m0] + snd:
        h.close()
    torch.cuda.synchronize()


for scheme in schemes:
    if scheme in ("prefilter", "prefilter_r05"):
        sim_prefilter(P, NW, r05=scheme == "prefilter_r05")
        continue
    if scheme == "prefilter_forest":
        sim_prefilter_forest(P, NW)
        continue
    ag = scheme == "allgather"       # replicated summaries: every rank folds every other rank's delta
    base = one_gpu_base(P, NW)
    ranks = [gsgpu.DisjointSet(V, id_bits=32, track_marks=(ag or r != 0), stream=torch.cuda.current_stream()) for r in range(P)]
    for h in ranks:
        h.timing(True)
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
            _, t = op(ranks[r], lambda: ranks[r].fold(s, d))
            fold_us.append(t)
        merge_us, xfer_us, npairs = 0.0, 0.0, []
        if ag:
            tex = []
            cnt_dev = torch.zeros(P, dtype=torch.int64, device="cuda")
            for r in range(P):
                _, te = op(ranks[r], lambda: ranks[r].export_marks_async(dbufs[r], cnt_dev[r:r + 1]))
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
                _, tf = op(ranks[r], lambda: fold_slots(ranks[r], rbuf[0], m, [0 if q == r else ns[q] for q in range(P)]) if m else None)
                ranks[r].set_marking(True)
                mt.append(tf)
            merge_us = max(mt)
            if os.environ.get("SIM_VERBOSE") and w < 3:
                print("   w%d deltas %s merge %s" % (w + 1, ns, ["%.0f" % x for x in mt]), flush=True)
        elif scheme == "gather":
            per = []
            for r in range(1, P):
                n, te = op(ranks[r], lambda: ranks[r].export_marks(buf))
                _, tf = op(ranks[0], lambda: ranks[0].fold_pairs(buf, n, id_bits=32))
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
                        n, te = op(ranks[r], lambda: ranks[r].export_marks(buf))
                        _, tf = op(ranks[peer], lambda: ranks[peer].fold_pairs(buf, n, id_bits=32))
                        npairs.append(n)
                        rnd_x = max(rnd_x, te + 8 * n / LINK * 1e6)
                        rnd_m = max(rnd_m, tf)
                xfer_us += rnd_x; merge_us += rnd_m
        close_us = []
        for r in range(P):
            _, t = op(ranks[r], lambda: ranks[r].close_window())
            close_us.append(t)
        crit = max(fold_us) + xfer_us + merge_us + (max(close_us) if ag else close_us[0]) + (GAP * 4 if KT else 0.0)
        tot["fold"] += max(fold_us); tot["close"] += close_us[0]; tot["crit"] += crit
        tot["xfer"] += xfer_us; tot["merge"] += merge_us; tot["pairs"] += sum(npairs)
        print("w%3d fold max %6.0f us (r0 %6.0f)  pairs %8d (max %7d)  xfer %6.0f  merge folds %6.0f  close r0 %5.0f  "
              "critical %6.0f us" % (w + 1, max(fold_us), fold_us[0], sum(npairs), max(npairs or [0]), xfer_us,
                                     merge_us, close_us[0], crit), flush=True)
    print("TOTAL %s: fold %.2f ms, xfer %.2f, merge %.2f, close %.2f, critical %.2f ms -> efficiency vs no-merge %.3f, "
          "pairs %d; one GPU %.2f ms -> model speedup %.2fx at P=%d"
          % (scheme, tot["fold"] / 1e3, tot["xfer"] / 1e3, tot["merge"] / 1e3, tot["close"] / 1e3,
             tot["crit"] / 1e3, (tot["fold"] + tot["close"]) / tot["crit"], tot["pairs"], base / 1e3,
             base / tot["crit"], P), flush=True)
    for r in ranks:
        r.close()
    torch.cuda.synchronize()
