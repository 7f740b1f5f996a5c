"""GPU parity of the production fold selection and of each named fold variant, one subprocess per
configuration (the library reads its debug variables once per process; csrc/cc_api.hip).

* test_headline_config_production: RMAT-26 EF16, 2^24-edge windows, production defaults — all 64
  windows bit-exact vs the C oracle's fixture (tests/golden/headline_rmat26.json), two back-to-back
  passes with reset, final labels vs an independent torch CC (tests/headline_check.py); the same
  with the reference's Long (int64) ids.
* test_headline_config_production[fold_windows]: the bench's timed call (gs_cc_fold_windows) over the
  whole stream in one call and in calls of 8 windows, each call's last window vs the fixture.
* test_c5_config_production: BASELINE config 5 (RMAT-24, 4,096 windows of 2^16 edges) — all 4,096
  windows vs the C oracle's fixture (tests/golden/c5_rmat24.json), per-window calls and the
  gs_cc_fold_windows path (one call; calls of 256 windows).
* test_headline_config_eight_ranks_one_gpu: the same stream as BASELINE config 3's 8-GPU strong
  layout (2^24-edge global windows, 2^21 edges per rank), 8 ranks through the C-ABI exchange on
  one GPU in allgather, gather and tree modes, all 64 windows vs the fixture
  (tests/headline_ranks_check.py).
* test_variant_parity: every golden stream, RMAT-21, ER-21 and the giant-switch stream, per window
  vs the C oracle, under production defaults and under each forced variant (tests/variant_check.py).
* test_fold_variants_verified: bench.py --verify (RMAT-22, 2^20-edge windows) under each variant.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _env(extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("GSGPU_")}
    env.update(extra)
    return env


def _last_json(out: bytes):
    return json.loads([l for l in out.decode().splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("args", [["--steps", "2"], ["--id-bits", "64", "--no-torch"], ["--fold-windows", "--no-torch"]],
                         ids=["int32_two_passes", "int64", "fold_windows"])
def test_headline_config_production(args):
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "headline_check.py")] + args, env=_env({}),
                                  timeout=900)
    r = _last_json(out)
    print(r)
    assert r["fixture_windows_equal"], r
    assert r["final_equals_torch_cc"] is not False and r["labels_minimal_idempotent"], r
    assert r["ok"], r


@pytest.mark.parametrize("args", [["--fold-windows", "--chunk", "256"], ["--id-bits", "64", "--no-torch"]],
                         ids=["int32_fold_windows", "int64"])
def test_c5_config_production(args):
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "headline_check.py"), "--fixture", "c5"] + args,
                                  env=_env({}), timeout=900)
    r = _last_json(out)
    print(r)
    assert r["windows"] == 4096 and r["fixture_windows_equal"], r
    assert r["ok"], r


def test_c5_latency_at_the_c_abi():
    """csrc/host/cc_latency (config 5 driven window by window from C++, no Python: what a Java FFM /
    JNI caller sees): the last window's emission equals the C oracle's fixture (window 4,096)."""
    exe = os.path.join(ROOT, "gelly-streaming_amd", "gsgpu", "lib", "cc_latency")
    out = subprocess.check_output([exe], env=_env({}), timeout=600)
    r = _last_json(out)
    print(r)
    fx = json.load(open(os.path.join(HERE, "golden", "c5_rmat24.json")))
    assert r["windows"] == 4096
    assert (int(r["final_checksum"]), r["final_vertices"], r["final_components"]) == \
        (int(fx["checksums"][-1]), int(fx["vertices"][-1]), int(fx["components"][-1]))


@pytest.mark.parametrize("mode", ["allgather", "gather", "tree", "prefilter"])
def test_headline_config_eight_ranks_one_gpu(mode):
    """BASELINE config 3's 8-rank strong layout at full scale through the C-ABI exchange
    (in-process transport): every window's emission vs the fixture, replicas equal, final vs torch CC."""
    args = ["--mode", mode] + ([] if mode == "allgather" else ["--no-torch"])
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "headline_ranks_check.py")] + args, env=_env({}),
                                  timeout=900)
    r = _last_json(out)
    print(r)
    assert not r["hung"] and not r["errors"], r
    assert r["fixture_windows_equal"] and r["replicas_equal"] and r["final_equals_torch_cc"] is not False, r


VARIANTS = {
    "production": {},
    # (the young split is off in production since round 5: forced here at capacity/16 = 2^17 for
    # the 2^21-id streams, as production ran it through round 4)
    "ring_warm_split_from_2^20": {"GSGPU_RING_MIN_BITS": "20", "GSGPU_YOUNG_SPLIT": str(1 << 17)},
    "ring_warm_no_split": {"GSGPU_RING_MIN_BITS": "20", "GSGPU_YOUNG_SPLIT": "0"},
    "ring_warm_stats": {"GSGPU_RING_MIN_BITS": "20", "GSGPU_FOLD_STATS": "1"},
    "ring_forced_no_warm": {"GSGPU_FOLD_MODE": "ring"},
    "plain_forced": {"GSGPU_FOLD_MODE": "plain", "GSGPU_RING_MIN_BITS": "20"},
    "young_split_2^18": {"GSGPU_YOUNG_SPLIT": str(1 << 18)},
    # no list-mode closes: every close after a logging fold is a bitmap or full one (the A/B knob
    # the round-4 list-close measurements ran against)
    "list_close_off": {"GSGPU_LIST_CLOSE": "0"},
}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_variant_parity(name):
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "variant_check.py")], env=_env(VARIANTS[name]),
                                  timeout=600)
    r = _last_json(out)
    bad = [c for c in r["cases"] if not c["ok"]]
    assert r["ok"] and not bad, bad


@pytest.mark.parametrize("name", ["production", "ring_warm_split_from_2^20", "plain_forced", "ring_warm_stats"])
def test_fold_variants_verified(name):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--scale", "22",
           "--edge-factor", "16", "--window-log2", "20", "--no-cpu-baseline", "--verify"]
    out = subprocess.check_output(cmd, env=_env(VARIANTS[name]), timeout=300)
    line = _last_json(out)
    assert line["verify"] == {"edges_consistent": True, "labels_minimal_idempotent": True, "equals_torch_cc": True}


@pytest.mark.parametrize("name", ["production", "list_close_off"])
def test_list_close_switch(name):
    """tests/test_gpu_listclose.py (list, bitmap and full closes mixed in one stream) and all 4,096
    windows of config 5 (RMAT-24, 2^16-edge windows: the list close's workload) with list-mode
    closes on (production) and off (GSGPU_LIST_CLOSE=0), each in a process of its own."""
    env = _env(VARIANTS[name])
    subprocess.check_call([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                           os.path.join(HERE, "test_gpu_listclose.py")], env=env, timeout=600, cwd=ROOT)
    out = subprocess.check_output([sys.executable, os.path.join(HERE, "headline_check.py"), "--fixture", "c5",
                                   "--fold-windows", "--chunk", "256"] + (["--variant"] if VARIANTS[name] else []),
                                  env=env, timeout=900)
    r = _last_json(out)
    assert r["windows"] == 4096 and r["fixture_windows_equal"] and r["ok"], r
