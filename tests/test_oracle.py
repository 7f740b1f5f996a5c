"""CPU: pin the oracle (C restatement + Python twin) against the reference's golden vectors."""
import ctypes
import json
import os

import numpy as np
import pytest

from pyoracle import (EMIT_CHECKSUM, EMIT_DENSE, PyDisjointSet, canonical_to_dense, dense_checksum,
                      py_cc_stream)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kats():
    with open(os.path.join(GOLD, "reference_kats.json")) as f:
        return json.load(f)


def _streams():
    with open(os.path.join(GOLD, "streams_index.json")) as f:
        idx = json.load(f)
    z = np.load(os.path.join(GOLD, "streams.npz"))   # allow_pickle=False (default)
    return [dict(c, **{k: z["%s__%s" % (c["name"], k)] for k in ("src", "dst", "labels", "checksums")})
            for c in idx]


# ---- DisjointSetTest (util/DisjointSetTest.java:37-78) ----
def test_disjointset_kat_python_twin():
    k = _kats()["DisjointSetTest"]
    ds = PyDisjointSet()
    for a, b in k["setup_unions"]:
        ds.union(a, b)
    assert len(ds.getMatches()) == k["expect_matches_size"]
    r0, r1 = ds.find(0), ds.find(1)
    assert r0 != r1
    for i in range(10):
        assert ds.find(i) == (r0 if i % 2 == 0 else r1)
    ds2 = PyDisjointSet()
    for a, b in k["merge_unions"]:
        ds2.union(a, b)
    ds2.merge(ds)
    assert len(ds2.getMatches()) == k["expect_merged_size"]
    assert len({ds2.find(e) for e in ds2.getMatches()}) == k["expect_merged_roots"]
    assert ds2.find(12345) is None                         # find() of an unknown id is null


def test_disjointset_kat_c_oracle(oracle):
    L = oracle.L
    k = _kats()["DisjointSetTest"]
    ds = L.gso_ds_new()
    for a, b in k["setup_unions"]:
        L.gso_ds_union(ds, a, b)
    assert L.gso_ds_size(ds) == k["expect_matches_size"]
    r = ctypes.c_int64()
    roots = []
    for i in range(10):
        assert L.gso_ds_find(ds, i, ctypes.byref(r)) == 1
        roots.append(r.value)
    assert roots[0] != roots[1]
    assert all(roots[i] == roots[i % 2] for i in range(10))
    ds2 = L.gso_ds_new()
    for a, b in k["merge_unions"]:
        L.gso_ds_union(ds2, a, b)
    L.gso_ds_merge(ds2, ds)
    assert L.gso_ds_size(ds2) == k["expect_merged_size"]
    rs = set()
    for i in range(L.gso_ds_size(ds2)):
        L.gso_ds_find(ds2, L.gso_ds_key_at(ds2, i), ctypes.byref(r))
        rs.add(r.value)
    assert len(rs) == k["expect_merged_roots"]
    assert L.gso_ds_find(ds2, 999, ctypes.byref(r)) == 0
    L.gso_ds_free(ds)
    L.gso_ds_free(ds2)


def test_combine_cc_merges_smaller_into_larger(oracle):
    L = oracle.L
    a, b = L.gso_ds_new(), L.gso_ds_new()
    L.gso_ds_union(a, 1, 2)
    for i in range(5):
        L.gso_ds_union(b, 10 + i, 11 + i)
    assert L.gso_combine(a, b) == b          # |a| = 2 <= |b| = 6 -> b.merge(a), return b
    assert L.gso_ds_size(b) == 8
    c = L.gso_ds_new()
    L.gso_ds_union(c, 100, 101)
    assert L.gso_combine(b, c) == b          # |b| = 8 > |c| = 2 -> b.merge(c), return b
    assert L.gso_ds_size(b) == 10
    for d in (a, b, c):
        L.gso_ds_free(d)


# ---- ConnectedComponentsTest (example/test/ConnectedComponentsTest.java:41,54-63) ----
def _components(labels: np.ndarray):
    comps = {}
    for v in np.nonzero(labels >= 0)[0].tolist():
        comps.setdefault(int(labels[v]), []).append(v)
    return sorted(", ".join(map(str, sorted(m))) for m in comps.values())


def test_connected_components_kat(oracle):
    k = _kats()["ConnectedComponentsTest"]
    e = np.array(k["edges"], dtype=np.int64)
    r = oracle.run(e[:, 0], e[:, 1], 0, partitions=1, emit=EMIT_DENSE, label_cap=16, want_final=True)
    assert _components(r["final"]) == k["expect_final_components"]
    # partition count does not change the result
    r4 = oracle.run(e[:, 0], e[:, 1], 2, partitions=4, emit=EMIT_DENSE, label_cap=16, want_final=True)
    assert _components(r4["final"]) == k["expect_final_components"]


def test_example_sample_stream(oracle):
    k = _kats()["ConnectedComponentsExample"]
    src = np.array(k["src"])
    dst = np.array(k["dst"])
    r = oracle.run(src, dst, 0, emit=EMIT_DENSE, label_cap=128, want_final=True)
    lab = r["final"]
    seen = np.nonzero(lab >= 0)[0]
    assert seen.size == k["expect_final_vertices"]
    assert all(lab[v] == (1 if v % 2 else 2) for v in seen)
    # event-time windows: cumulative emissions after each window
    for w in k["event_time_windows"]:
        a, b = w["edges"]
        rr = oracle.run(src[:b], dst[:b], 0, emit=EMIT_DENSE, label_cap=128, want_final=True)
        assert int((rr["final"] >= 0).sum()) == w["n_vertices"]


# ---- seeded streams: per-window emissions ----
@pytest.mark.parametrize("case", _streams(), ids=lambda c: c["name"])
def test_streams_golden_c_oracle(oracle, case):
    r = oracle.run(case["src"], case["dst"], case["window_edges"], partitions=case["partitions"],
                   threads=2, emit=EMIT_DENSE, label_cap=case["cap"])
    assert r["windows"] == case["labels"].shape[0]
    np.testing.assert_array_equal(r["labels"], case["labels"])
    np.testing.assert_array_equal(r["checksums"], case["checksums"])
    for w in range(r["windows"]):
        assert dense_checksum(case["labels"][w])[0] == int(case["checksums"][w])


@pytest.mark.parametrize("case", _streams(), ids=lambda c: c["name"])
def test_run_from_restored_merger(oracle, case):
    """gso_cc_run_from: the Merger restored from window k's canonical emission (restoreState,
    SummaryAggregation.java:127-135) continues the stream with the uninterrupted emissions."""
    W, nwin = case["window_edges"], case["labels"].shape[0]
    k = nwin // 2
    if k == 0:
        pytest.skip("one window")
    lab = case["labels"][k - 1]
    v = np.nonzero(lab >= 0)[0].astype(np.int64)
    r = oracle.run(case["src"][k * W:], case["dst"][k * W:], W, partitions=case["partitions"], threads=2,
                   emit=EMIT_DENSE, label_cap=case["cap"], init=(v, lab[v]))
    np.testing.assert_array_equal(r["labels"], case["labels"][k:])


@pytest.mark.parametrize("case", _streams()[:4], ids=lambda c: c["name"])
def test_streams_golden_python_twin(case):
    emis = py_cc_stream(case["src"].tolist(), case["dst"].tolist(), case["window_edges"], case["partitions"])
    for w, c in enumerate(emis):
        np.testing.assert_array_equal(canonical_to_dense(c, case["cap"]), case["labels"][w])


@pytest.mark.parametrize("P,W", [(1, 1000), (3, 777), (8, 4096), (5, 0)])
def test_partition_and_window_invariance_of_final_labels(oracle, P, W):
    s, d = oracle.gen_rmat(0, 20000, 12, 3)
    base = oracle.run(s, d, 0, partitions=1, emit=EMIT_CHECKSUM, label_cap=4096, want_final=True)
    r = oracle.run(s, d, W, partitions=P, threads=4, emit=EMIT_CHECKSUM, label_cap=4096, want_final=True)
    np.testing.assert_array_equal(base["final"], r["final"])
    assert r["final_vertices"] == base["final_vertices"]


def test_checksum_definition_c_matches_numpy(oracle):
    lab = np.array([-1, 0, 0, 3, -1, 3, 0], dtype=np.int64)
    want = 0
    for v, l in enumerate(lab.tolist()):
        if l >= 0:
            want = (want + oracle.L.gso_pair_mix(v, l)) & ((1 << 64) - 1)
    assert dense_checksum(lab)[0] == want


# ---- generators ----
def test_generators_golden(oracle):
    with open(os.path.join(GOLD, "generators.json")) as f:
        g = json.load(f)
    s, d = oracle.gen_rmat(0, 64, 20, 1)
    assert [s.tolist(), d.tolist()] == g["rmat_s20_seed1_first0"]
    s, d = oracle.gen_rmat(1 << 20, 64, 26, 1)
    assert [s.tolist(), d.tolist()] == g["rmat_s26_seed1_first1M"]
    s, d = oracle.gen_er(0, 64, 1 << 24, 2)
    assert [s.tolist(), d.tolist()] == g["er_n2^24_seed2_first0"]
    s, d = oracle.gen_rmat(5, 64, 12, 9, scramble=False)
    assert [s.tolist(), d.tolist()] == g["rmat_s12_seed9_first5_noscramble"]


def test_generator_is_counter_based(oracle):
    s, d = oracle.gen_rmat(0, 1000, 16, 5)
    s2, d2 = oracle.gen_rmat(400, 600, 16, 5)
    np.testing.assert_array_equal(s[400:], s2)
    np.testing.assert_array_equal(d[400:], d2)
    assert s.min() >= 0 and s.max() < (1 << 16)


def test_rmat_scramble_is_bijection(oracle):
    # scrambled ids of the unscrambled stream's distinct ids stay distinct
    s, d = oracle.gen_rmat(0, 50000, 10, 11, scramble=False)
    s2, d2 = oracle.gen_rmat(0, 50000, 10, 11, scramble=True)
    pairs = {}
    for a, b in zip(np.concatenate([s, d]).tolist(), np.concatenate([s2, d2]).tolist()):
        assert pairs.setdefault(a, b) == b
    assert len(set(pairs.values())) == len(pairs)


def test_oracle_under_host_sanitizers():
    """The checker itself is clean under AddressSanitizer + UBSan (oracle/sanitize_main.c)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "check-asan"], capture_output=True,
                         timeout=300)
    assert out.returncode == 0, out.stdout.decode() + out.stderr.decode()
    assert b"sanitizer run OK" in out.stdout


def test_headline_fixture_window1_live(oracle):
    """tests/golden/headline_rmat26.json (minted by tests/golden/make_headline.py with P = 8) agrees with
    a live oracle run of window 1 of the headline stream at another partition count (P = 3): the
    emission is independent of P, and the fixture is what the checker computes."""
    fx = json.load(open(os.path.join(GOLD, "headline_rmat26.json")))
    assert fx["windows"] == 64 and len(fx["checksums"]) == 64
    assert fx["vertices"] == sorted(fx["vertices"]) and fx["vertices"][-1] <= 1 << fx["scale"]
    W = fx["window_edges"]
    s, d = oracle.gen_rmat(0, W, fx["scale"], fx["seed"])
    r = oracle.run(s, d, W, partitions=3, threads=3, emit=EMIT_CHECKSUM)
    assert int(r["checksums"][0]) == int(fx["checksums"][0])
    assert [int(x) for x in r["counts"][0]] == [fx["vertices"][0], fx["components"][0]]


@pytest.mark.parametrize("kind,param,n,W,seed", [("rmat", 16, 1 << 20, 1 << 12, 3), ("er", 1 << 16, 1 << 17, 1 << 10, 2),
                                                 ("rmat", 12, 1 << 16, 333, 5)])
def test_emission_tracker_matches_full_checksum(oracle, kind, param, n, W, seed):
    """oracle/emission.c (GSO_EMIT_TRACK, used to mint the 4,096-window config-5 fixture) gives the
    same per-window checksum, vertex and component counts as the full canonical checksum of the
    Merger's summary (gso_ds_canonical_checksum) on every window; its own cross-check runs too."""
    from pyoracle import EMIT_TRACK
    s, d = oracle.gen_rmat(0, n, param, seed) if kind == "rmat" else oracle.gen_er(0, n, param, seed)
    cap = (1 << param) if kind == "rmat" else param
    a = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_CHECKSUM, label_cap=cap)
    b = oracle.run(s, d, W, partitions=4, threads=4, emit=EMIT_TRACK, label_cap=cap, verify_every=7)
    np.testing.assert_array_equal(a["checksums"], b["checksums"])
    np.testing.assert_array_equal(a["counts"], b["counts"])


def test_c5_fixture_first_windows_live(oracle):
    """tests/golden/c5_rmat24.json (tracker, P = 8) agrees with a live full-checksum oracle run of its
    first 32 windows at another partition count (P = 3), and its counts are monotone."""
    fx = json.load(open(os.path.join(GOLD, "c5_rmat24.json")))
    assert fx["windows"] == 4096 and len(fx["checksums"]) == 4096 and fx["window_edges"] == 1 << 16
    assert fx["vertices"] == sorted(fx["vertices"]) and fx["vertices"][-1] <= 1 << fx["scale"]
    W, k = fx["window_edges"], 32
    s, d = oracle.gen_rmat(0, k * W, fx["scale"], fx["seed"])
    r = oracle.run(s, d, W, partitions=3, threads=3, emit=EMIT_CHECKSUM)
    assert [int(x) for x in r["checksums"]] == [int(x) for x in fx["checksums"][:k]]
    assert [int(x) for x in r["counts"][:, 0]] == fx["vertices"][:k]
    assert [int(x) for x in r["counts"][:, 1]] == fx["components"][:k]


# ---------------- edge-file input (oracle/parse.c) vs the Java rules ----------------
def _java_split_parse(text: bytes):
    """ConnectedComponentsExample.java:108-119 with Python's re: line.split("\\\\s") (trailing
    empties dropped), Long.parseLong of fields 0 and 1; (src, dst) or the first bad line index."""
    import re
    lines = text.decode().split("\n")
    if lines and lines[-1] == "":
        lines = lines[:-1]
    src, dst = [], []
    for i, ln in enumerate(lines):
        f = re.split(r"[ \t\n\x0b\f\r]", ln)
        while f and f[-1] == "":
            f.pop()
        ok = len(f) >= 2 and all(re.fullmatch(r"[+-]?[0-9]+", x) for x in f[:2])
        if ok:
            a, b = int(f[0]), int(f[1])
            ok = -(1 << 63) <= a < (1 << 63) and -(1 << 63) <= b < (1 << 63)
        if not ok:
            return i
        src.append(a)
        dst.append(b)
    return np.array(src, dtype=np.int64), np.array(dst, dtype=np.int64)


def test_oracle_parse_edges_valid_forms(oracle):
    text = (b"1 2\n3\t4\n5 6 extra fields\n+7 -8\r\n9 10  \n-9223372036854775808 9223372036854775807\n" +
            b"".join(b"%d %d\n" % (i, i * 7 % 1000) for i in range(5000)) + b"11 12")
    want = _java_split_parse(text)
    s, d, _ = oracle.parse_edges(text)
    np.testing.assert_array_equal(s, want[0])
    np.testing.assert_array_equal(d, want[1])


@pytest.mark.parametrize("bad", [b"1  2\n", b"\n", b" 1 2\n", b"1x 2\n", b"1\n", b"1 99999999999999999999\n",
                                 b"1 9223372036854775808\n", b"- 3\n", b"   \n"])
def test_oracle_parse_edges_rejects_what_java_rejects(oracle, bad):
    text = b"5 6\n7 8\n" + bad + b"9 10\n"
    assert _java_split_parse(text) == 2
    assert oracle.parse_edges(text)[0] == 2


def test_oracle_parse_edges_random(oracle):
    s, d = oracle.gen_rmat(0, 20000, 20, 5)
    text = "".join("%d %d\n" % (a, b) for a, b in zip(s.tolist(), d.tolist())).encode()
    ps, pd, _ = oracle.parse_edges(text)
    np.testing.assert_array_equal(ps, s)
    np.testing.assert_array_equal(pd, d)
