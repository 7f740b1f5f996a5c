"""Measured HBM copy peak on the box (report a measured STREAM-copy figure beside
the 8 TB/s spec peak). Device-to-device copy of a 4 GiB buffer, bytes = read + write, HIP events
around 20 copies after 3 warmups. Prints one JSON line. usage: python tools/hbm_peak.py"""
import json

import torch


def main():
    n = 1 << 30                                   # 4 GiB of int32
    src = torch.ones(n, dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = 2 * 4 * n / (ms * 1e-3) / 1e9
    print(json.dumps({"what": "d2d copy 4 GiB, read+write bytes", "ms_per_copy": ms, "GB_per_s": gbs,
                      "spec_peak_GB_per_s": 8000.0, "device": torch.cuda.get_device_name(0)}))


if __name__ == "__main__":
    main()
