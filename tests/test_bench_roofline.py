"""bench.py's request roofline (CPU): it is computed from the committed PMC counts and the committed
request-rate lab, and stays consistent with both."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def _args(**kw):
    sys.argv = ["bench.py"] + [x for k, v in kw.items() for x in ("--" + k.replace("_", "-"), str(v))]
    import bench
    return bench, bench.parse()


def test_request_roofline_from_committed_counts():
    bench, a = _args()
    W = 1 << a.window_log2
    r = bench.request_roofline(a, W, 0.2226)
    assert r is not None and r["bound"] == "l2-requests"
    tj = json.load(open(os.path.join(ROOT, "profiles", "fold_traffic.json")))
    lab = json.load(open(os.path.join(ROOT, "profiles", "r02_request_lab.json")))
    ring = tj["ring"]
    assert abs(r["l2_hits_per_launch"] + r["l2_misses_per_launch"] - ring["tcc_requests_per_launch"]) < 1.0
    assert r["hit_rate_peak_Gps"] == lab["rand4B_1MiB_32w_Gps"]
    assert r["miss_rate_peak_Gps"] == lab["rand4B_64MiB_32w_Gps"]
    # the bound is the slower of the two paths, and below the measured launch time
    assert r["bound_us"] == max(r["hits_us"], r["misses_us"])
    assert 0.0 < r["frac"] < 1.0
    assert abs(r["frac"] - r["bound_us"] / 222.6) < 1e-9
    # the lab's ordering: L2-resident > Infinity Cache >= HBM for random 4-B loads
    assert lab["rand4B_1MiB_32w_Gps"] > lab["rand4B_8MiB_32w_Gps"] > lab["rand4B_64MiB_32w_Gps"] >= lab["rand4B_2GiB_32w_Gps"]


def test_request_roofline_only_for_the_counted_configuration():
    bench, a = _args(window_log2=21)
    assert bench.request_roofline(a, 1 << 21, 0.05) is None     # counts were taken on 2^24-edge windows
