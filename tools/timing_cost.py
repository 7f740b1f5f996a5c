"""Wall time of the headline step (RMAT-26, 64 windows) with and without the per-launch HIP
timing events bench.py attaches (what the events cost)."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import gsgpu
from gsgpu import gen
scale, W, nwin = 26, 1 << 24, 64
V = 1 << scale
s = torch.empty(nwin * W, dtype=torch.int32, device="cuda"); d = torch.empty(nwin * W, dtype=torch.int32, device="cuda")
for w in range(nwin):
    gen.rmat(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W], w * W, scale, 1)
ds = gsgpu.DisjointSet(V, id_bits=32, stream=torch.cuda.current_stream())
def step():
    ds.reset()
    for w in range(nwin):
        ds.fold(s[w * W:(w + 1) * W], d[w * W:(w + 1) * W]); ds.close_window()
from gsgpu._abi import GS_TIMING_MASK, GS_K_FOLD
for timing in (False, True, GS_TIMING_MASK | (1 << GS_K_FOLD), False, True, GS_TIMING_MASK | (1 << GS_K_FOLD)):
    ds.timing(timing)
    step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    print("timing %-5s %.3f ms/step" % (timing, (time.perf_counter() - t0) / 3 * 1e3), flush=True)
