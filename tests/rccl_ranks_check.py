"""The C-ABI exchange over REAL RCCL with several ranks, on one GPU: one process per rank.

RCCL refuses two ranks of one communicator on one device when it sees them on one host ("Duplicate
GPU detected"). Each rank process here gets its own NCCL_HOSTID, so RCCL takes the ranks for
separate hosts and connects them through its network transport over the loopback interface
(NCCL_SOCKET_IFNAME=lo) instead of P2P / SHM. The exchange code is the production one: the
prefilter's ncclBroadcast of the filter state (and the ncclCommSplit side communicator its
asynchronous broadcasts use), its count-headed ncclSend/ncclRecv survivor slots, the all-gather's
speculative slots with lazy verification, the gather and the tree rounds (csrc/comm.hip). The
timings of this transport mean nothing; the emissions must be exact.

  python tests/rccl_ranks_check.py --world 4           # launcher: oracle, P rank processes, checks
  (the launcher starts `--rank r` children itself)

Checks, one JSON line from the launcher: in every mode, the checked ranks' emission checksum after
EVERY window equals the C oracle's (tests only: the oracle is the checker), and their final dense
labels equal the oracle's (allgather: every rank is a replica of the Merger; gather / tree /
prefilter: rank 0); then allgather / gather / tree once more with sparse int64 ids (negative ids,
INT64_MIN / MAX: the reference's Long keys), whose exchange carries 16-B (id, root id) pairs.
Reference: SummaryBulkAggregation.java:76-83 (partitions -> windowAll -> Merger),
SummaryTreeReduce.java:95-123 (the tree), SummaryAggregation.java:106-119 (emission).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

MODES = ("allgather", "gather", "tree", "prefilter")
SPARSE_MODES = ("allgather", "gather", "tree")      # (prefilter: dense ids only)


def _wait_file(path: str, timeout: float = 120.0) -> bytes:
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout:
            raise TimeoutError(path)
        time.sleep(0.02)
    with open(path, "rb") as f:
        return f.read()


def _put_file(path: str, data: bytes) -> None:
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def rank_main(a) -> int:
    import numpy as np
    import torch
    import gsgpu
    from gsgpu import Comm
    from gsgpu.comm import unique_id
    from variant_check import rank_slices
    assert torch.cuda.is_available(), "needs a HIP device"
    r, P, W, cap = a.rank, a.world, a.window, a.cap
    s = np.load(os.path.join(a.dir, "src.npy"))
    d = np.load(os.path.join(a.dir, "dst.npy"))
    ts = torch.from_numpy(s.astype(np.int32)).cuda()
    td = torch.from_numpy(d.astype(np.int32)).cuda()
    out = {"rank": r, "modes": {}}
    for mode in MODES:
        uid_path = os.path.join(a.dir, "uid_%s.bin" % mode)
        if r == 0:
            _put_file(uid_path, unique_id())
        comm = Comm.create(_wait_file(uid_path), r, P, 0)
        pre = mode == "prefilter"
        sl = rank_slices(s.size, W, P, a.share0 if pre else None)[r]
        ds = gsgpu.DisjointSet(cap, id_bits=32, track_marks=not pre)
        sums = []
        t0 = time.time()
        for lo, hi in sl:
            if pre:
                assert ds.fold_windows(ts[lo:hi], td[lo:hi], max(hi - lo, 1), comm=comm, mode="prefilter") == 1
            else:
                ds.fold(ts[lo:hi], td[lo:hi])
                ds.merge_window(comm, mode)
            if r == 0 or mode == "allgather":
                sums.append(int(ds.checksum()[0]))
        rec = {"checksums": sums, "seconds": round(time.time() - t0, 2), "info": list(comm.info())}
        if r == 0 or mode == "allgather":
            np.save(os.path.join(a.dir, "final_%s_%d.npy" % (mode, r)), ds.dense().astype(np.int64))
        ds.close()
        comm.close()
        out["modes"][mode] = rec
    # sparse int64 ids (any Long key): the exchange carries (id, root id) 16-B pairs
    ss = torch.from_numpy(np.load(os.path.join(a.dir, "ssrc.npy"))).cuda()
    sd = torch.from_numpy(np.load(os.path.join(a.dir, "sdst.npy"))).cuda()
    for mode in SPARSE_MODES:
        uid_path = os.path.join(a.dir, "uid_sparse_%s.bin" % mode)
        if r == 0:
            _put_file(uid_path, unique_id())
        comm = Comm.create(_wait_file(uid_path), r, P, 0)
        ds = gsgpu.DisjointSet(a.sparse_cap, id_bits=64, track_marks=True, sparse=True)
        sums = []
        for lo, hi in rank_slices(ss.numel(), a.sparse_window, P)[r]:
            ds.fold(ss[lo:hi], sd[lo:hi])
            ds.merge_window(comm, mode)
            if r == 0 or mode == "allgather":
                sums.append([int(x) for x in ds.checksum()])
        ds.close()
        out["modes"]["sparse_" + mode] = {"checksums": sums, "seconds": 0.0, "info": list(comm.info())}
        comm.close()
    with open(os.path.join(a.dir, "rank%d.json" % r), "w") as f:
        json.dump(out, f)
    return 0


def launch_main(a) -> int:
    import numpy as np
    from pyoracle import EMIT_CHECKSUM, coracle
    oracle = coracle()
    cap = 1 << a.scale
    s, d = oracle.gen_rmat(0, a.edges, a.scale, a.seed)
    want = oracle.run(s, d, a.window, partitions=a.world, threads=4, emit=EMIT_CHECKSUM, label_cap=cap,
                      want_final=True)
    ws = [int(x) for x in want["checksums"]]
    ss, sd = oracle.gen_rmat(0, a.sparse_edges, 14, a.seed + 1)
    mul = np.uint64(0x9E3779B97F4A7C15)                   # odd: an injective map over the int64 range
    with np.errstate(over="ignore"):
        ss = (ss.astype(np.uint64) * mul).view(np.int64)
        sd = (sd.astype(np.uint64) * mul).view(np.int64)
    ss[:3] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, -1]
    sd[:3] = [-1, 5, np.iinfo(np.int64).min]
    swant = oracle.run(ss, sd, a.sparse_window, partitions=a.world, emit=EMIT_CHECKSUM)
    sexp = [[int(c), int(v), int(k)] for c, (v, k) in zip(swant["checksums"], swant["counts"])]
    t0 = time.time()
    res = {"world": a.world, "scale": a.scale, "edges": a.edges, "window": a.window, "windows": len(ws),
           "transport": "RCCL net (sockets over lo), one process per rank, distinct NCCL_HOSTID"}
    with tempfile.TemporaryDirectory(prefix="gs_rccl_") as tmp:
        np.save(os.path.join(tmp, "src.npy"), s)
        np.save(os.path.join(tmp, "dst.npy"), d)
        np.save(os.path.join(tmp, "ssrc.npy"), ss)
        np.save(os.path.join(tmp, "sdst.npy"), sd)
        procs = []
        for r in range(a.world):
            env = dict(os.environ)
            env.update({"NCCL_HOSTID": "gsgpu-rccl-rank%d" % r, "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                        "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
            cmd = [sys.executable, "-u", os.path.abspath(__file__), "--rank", str(r), "--world", str(a.world),
                   "--dir", tmp, "--window", str(a.window), "--cap", str(cap), "--share0", str(a.share0),
                   "--sparse-window", str(a.sparse_window), "--sparse-cap", str(a.sparse_cap)]
            procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        rcs, logs = [], []
        deadline = time.time() + a.timeout
        for p in procs:
            try:
                o, _ = p.communicate(timeout=max(1.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                for q in procs:
                    if q.poll() is None:
                        q.kill()
                o, _ = p.communicate()
                rcs.append("timeout")
                logs.append(o[-3000:])
                continue
            rcs.append(p.returncode)
            logs.append(o[-3000:] if p.returncode else "")
        res["returncodes"] = rcs
        if any(rc != 0 for rc in rcs):
            res["ok"] = False
            res["logs"] = logs
            print(json.dumps(res), flush=True)
            return 1
        ranks = []
        for r in range(a.world):
            with open(os.path.join(tmp, "rank%d.json" % r)) as f:
                ranks.append(json.load(f))
        modes = {}
        ok = True
        for mode in MODES:
            checked = list(range(a.world)) if mode == "allgather" else [0]
            m = {"checked_ranks": checked, "seconds": [ranks[r]["modes"][mode]["seconds"] for r in range(a.world)],
                 "bytes_sent": [ranks[r]["modes"][mode]["info"][2] for r in range(a.world)],
                 "bytes_recv": [ranks[r]["modes"][mode]["info"][3] for r in range(a.world)],
                 "overflow_rounds": [ranks[r]["modes"][mode]["info"][5] for r in range(a.world)]}
            first_bad = {}
            for r in checked:
                got = ranks[r]["modes"][mode]["checksums"]
                bad = next((w for w in range(len(ws)) if w >= len(got) or got[w] != ws[w]), None)
                if len(got) != len(ws) and bad is None:
                    bad = len(ws)
                fin = np.load(os.path.join(tmp, "final_%s_%d.npy" % (mode, r)))
                if not np.array_equal(fin, want["final"]):
                    bad = "final" if bad is None else bad
                first_bad[r] = bad
            m["first_bad_window"] = first_bad
            # data crossed the wire between processes (a sender sent, rank 0 received)
            m["peers_exchanged"] = bool(sum(m["bytes_recv"]) > 0 and sum(m["bytes_sent"][1:]) > 0)
            m["ok"] = all(v is None for v in first_bad.values()) and m["peers_exchanged"]
            ok &= m["ok"]
            modes[mode] = m
        for mode in SPARSE_MODES:
            checked = list(range(a.world)) if mode == "allgather" else [0]
            recs = [ranks[r]["modes"]["sparse_" + mode] for r in range(a.world)]
            first_bad = {}
            for r in checked:
                got = recs[r]["checksums"]
                first_bad[r] = next((w for w in range(len(sexp)) if w >= len(got) or got[w] != sexp[w]), None)
            m = {"checked_ranks": checked, "ids": "sparse int64 (16-B pairs)",
                 "bytes_recv": [x["info"][3] for x in recs], "first_bad_window": first_bad,
                 "peers_exchanged": sum(x["info"][3] for x in recs) > 0}
            m["ok"] = all(v is None for v in first_bad.values()) and m["peers_exchanged"]
            ok &= m["ok"]
            modes["sparse_" + mode] = m
        res["modes"] = modes
    res["ok"] = bool(ok)
    res["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


def main() -> int:
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--rank", type=int, default=-1, help="(internal) run as this rank")
    ap.add_argument("--dir", default="")
    ap.add_argument("--scale", type=int, default=16)
    ap.add_argument("--edges", type=int, default=240000)
    ap.add_argument("--window", type=int, default=8000)
    ap.add_argument("--cap", type=int, default=0)
    ap.add_argument("--share0", type=float, default=0.125)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--sparse-edges", type=int, default=120000)
    ap.add_argument("--sparse-window", type=int, default=20000)
    ap.add_argument("--sparse-cap", type=int, default=1 << 15)
    ap.add_argument("--timeout", type=float, default=240.0)
    a = ap.parse_args()
    return rank_main(a) if a.rank >= 0 else launch_main(a)


if __name__ == "__main__":
    sys.exit(main())
