"""The exchange over real RCCL between rank PROCESSES (tests/rccl_ranks_check.py): every mode's
emission after every window vs the C oracle, with data crossing between processes — the
prefilter's broadcasts (synchronous, and asynchronous over the split communicator) and
send/recv slots, the all-gather's speculative slots, the gather and the tree rounds. One GPU:
each rank process has its own NCCL_HOSTID, so RCCL connects them through its network transport
over loopback (it refuses two same-host ranks on one device)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_rank_processes_every_mode_vs_oracle(world):
    cmd = [sys.executable, "-u", os.path.join(HERE, "rccl_ranks_check.py"), "--world", str(world)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=420)
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert lines, (out.returncode, out.stdout[-3000:], out.stderr[-3000:])
    r = json.loads(lines[-1])
    assert r["ok"] and out.returncode == 0, r
    for mode, m in r["modes"].items():
        assert m["peers_exchanged"], (mode, m)


@pytest.mark.parametrize("merge", ["prefilter", "allgather", "gather", "tree"])
def test_bench_rank_processes_over_rccl(merge):
    """The driver's N > 1 bench path (bench.py under torch.distributed, RCCL for torch's process group
    and for the C-ABI exchange), two rank processes on this GPU (tools/bench_ranks_one_gpu.py):
    both exit 0 and rank 0's final labels equal an independent torch CC of the whole stream."""
    root = os.path.dirname(HERE)
    cmd = [sys.executable, "-u", os.path.join(root, "tools", "bench_ranks_one_gpu.py"), "--ranks", "2", "--timeout", "300",
           "--", "--scale", "20", "--window-log2", "18", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
           "--verify", "--merge", merge]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=360)
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert lines, (out.returncode, out.stdout[-3000:], out.stderr[-3000:])
    r = json.loads(lines[-1])
    assert r["ok"] and out.returncode == 0, r
    b = r["bench_line"]
    assert b["n_gpus"] == 2 and b["exchange"]["merge"] == merge, b
    assert b["verify"]["equals_torch_cc"], b["verify"]
