"""Rehearse the driver's N > 1 bench path (bench.py under torch.distributed, RCCL for torch's process
group AND for the C-ABI exchange) on ONE GPU: P bench.py rank processes with the env torchrun would
give them (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT), each with its own NCCL_HOSTID so RCCL
takes them for separate hosts and connects them through its network transport over loopback
(it refuses two same-host ranks on one device). bench.py maps LOCAL_RANK onto the one device
(`local % device_count`).

The timings of this transport (host sockets, P ranks sharing one GPU) mean nothing; what this
checks is that the multi-rank bench runs end to end over RCCL and that rank 0's timed emission
equals the fixture (`final_checksum_vs_fixture`) and, with --verify, an independent torch CC.

  python tools/bench_ranks_one_gpu.py --ranks 4 -- --steps 1 --warmup 0 --no-cpu-baseline --verify
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main() -> int:
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--log-dir", default="", help="write every rank's stderr there (rank<r>.err)")
    a = ap.parse_args(argv)
    port = free_port()
    procs = []
    t0 = time.time()
    for r in range(a.ranks):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(a.ranks), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(a.ranks),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "NCCL_HOSTID": "gsgpu-bench-rank%d" % r, "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(a.ranks)] + extra
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs, rcs = [], []
    deadline = time.time() + a.timeout
    for p in procs:
        try:
            o, e = p.communicate(timeout=max(1.0, deadline - time.time()))
            rcs.append(p.returncode)
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            o, e = p.communicate()
            rcs.append("timeout")
        outs.append((o, e))
    if a.log_dir:
        os.makedirs(a.log_dir, exist_ok=True)
        for r, (_, e) in enumerate(outs):
            with open(os.path.join(a.log_dir, "rank%d.err" % r), "w") as f:
                f.write(e)
    line = None
    for ln in outs[0][0].splitlines():
        if ln.startswith("{"):
            line = json.loads(ln)
    res = {"ranks": a.ranks, "returncodes": rcs, "seconds": round(time.time() - t0, 1),
           "transport": "RCCL net (sockets over lo), P processes on one GPU: timings not meaningful",
           "bench_line": line}
    if line is None or any(rc != 0 for rc in rcs):
        res["stderr_tails"] = [e[-2500:] for _, e in outs]
    ok = line is not None and all(rc == 0 for rc in rcs)
    if line is not None:
        fx = line.get("final_checksum_vs_fixture") or {}
        ok = ok and fx.get("match", True) is not False
        ver = line.get("verify")
        if isinstance(ver, dict):
            ok = ok and all(v is not False for v in ver.values())
    res["ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
