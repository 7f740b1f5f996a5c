"""bench.py's roofline figures (CPU): every committed bench line of this round has a sane fraction
computed from the edges each launch actually folded, and PMC-derived figures are used only when
the committed profile was measured on the same kernel sources."""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))


def _bench(**kw):
    sys.argv = ["bench.py"] + [x for k, v in kw.items() for x in ("--" + k.replace("_", "-"), str(v))]
    import bench
    return bench, bench.parse()


def _lines():
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0[34]_*bench*.json"))):
        for ln in open(f):
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                out.append((f, json.loads(ln)))
    return out


def test_committed_lines_have_sane_fractions():
    lines = _lines()
    for f, d in lines:
        r = d["roofline"]
        if str(d["config"].get("workload", "")).startswith(("parse", "bip")):   # SURVEY 8(f) rows (bench_rows.py)
            assert 0.0 < r["frac"] <= 1.0 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9, f
            assert d["verify"] and all(v is True for k, v in d["verify"].items() if isinstance(v, bool)), f
            assert d["cpu_baseline"]["value"] > 0, f
            continue
        per_edge = 16 if d["config"]["id_bits"] == 32 else 32
        assert 0.0 < r["frac"] <= 1.0, (f, r["frac"])
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9, f
        assert r["edges_per_launch"] <= (1 << 24), f                 # the library's internal cut
        assert abs(r["alg_bytes_per_launch"] - per_edge * r["edges_per_launch"]) < 1e-6, f
        assert 0.0 < (r.get("step") or r["wall"])["frac"] <= 1.0, f   # round 3's lines: "wall"
        assert 0.0 < r["fold_all"]["frac"] <= 1.0, f
        if r.get("requests"):
            assert 0.0 < r["requests"]["frac"] <= 1.0, f


def test_stale_profile_is_dropped(tmp_path):
    from gsgpu._abi import lib_source_sha
    bench, a = _bench()
    prof = {"lib_source_sha": "0" * 16, "scale": a.scale, "id_bits": 32,
            "steady": {"kernel": "k_fold_ring", "edges_per_launch": 1 << 24, "hbm_bytes_per_launch": 1e8,
                       "tcc_requests_per_launch": 1e7}}
    p = tmp_path / "t.json"
    p.write_text(json.dumps(prof))
    a.traffic_json = str(p)
    st, note = bench.steady_profile(a, "k_fold_ring", 1 << 24)
    assert st is None and note.startswith("stale")
    prof["lib_source_sha"] = lib_source_sha()
    p.write_text(json.dumps(prof))
    st, note = bench.steady_profile(a, "k_fold_ring", 1 << 24)
    assert st is not None and st["hbm_bytes_per_launch"] == 1e8
    st, note = bench.steady_profile(a, "k_fold", 1 << 24)               # another kernel: not used
    assert st is None
    st, note = bench.steady_profile(a, "k_fold_ring", 1 << 21)       # another launch size: not used
    assert st is None


def test_request_roofline_definition():
    bench, a = _bench()
    lab = json.load(open(os.path.join(ROOT, "profiles", "r03_request_lab.json")))
    prof = {"tcc_requests_per_launch": 13.0e6, "hbm_bytes_per_launch": 400e6}
    r = bench.request_roofline(prof, 0.1)
    t_req = 13.0e6 / (lab["rand4B_1MiB_32w_Gps"] * 1e3)
    t_b = 400e6 / (lab["stream_read_TBps"] * 1e6)
    assert abs(r["bound_us"] - max(t_req, t_b)) < 1e-9
    assert abs(r["frac"] - r["bound_us"] / 100.0) < 1e-9
    assert r["bound"] == ("l2-requests" if t_req >= t_b else "hbm-bytes")
    # the lab's ordering: L2-resident > Infinity Cache >= HBM for random 4-B loads
    assert lab["rand4B_1MiB_32w_Gps"] > lab["rand4B_8MiB_32w_Gps"] > lab["rand4B_64MiB_32w_Gps"] >= lab["rand4B_2GiB_32w_Gps"]


def test_request_roofline_miss_term():
    """With the L2 hit rate in the profile, the misses go to the fabric at the lab's random-miss rate
    (64 MiB table); the bound is the largest of the three terms."""
    bench, a = _bench()
    lab = json.load(open(os.path.join(ROOT, "profiles", "r03_request_lab.json")))
    prof = {"tcc_requests_per_launch": 34.85e6, "hbm_bytes_per_launch": 636e6, "l2_hit_rate": 0.74}
    r = bench.request_roofline(prof, 0.22)
    t_req = 34.85e6 / (lab["rand4B_1MiB_32w_Gps"] * 1e3)
    t_miss = 34.85e6 * 0.26 / (lab["rand4B_64MiB_32w_Gps"] * 1e3)
    t_b = 636e6 / (lab["stream_read_TBps"] * 1e6)
    assert abs(r["l2_misses_per_launch"] - 34.85e6 * 0.26) < 1.0
    assert abs(r["bound_us"] - max(t_req, t_miss, t_b)) < 1e-9
    assert r["bound"] == "l2-misses" and t_miss > t_req
    assert abs(r["frac"] - r["bound_us"] / 220.0) < 1e-9
