"""bench.py's SURVEY.md 8(f) lines end to end at small sizes: edge-file ingestion parses the text of
a generated stream back into exactly its ids (and the C oracle parses the same text), and
BipartitenessCheck on a bipartite stream stays bipartite with the component counts of the CC path."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra):
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1"]
                                  + list(extra), timeout=300).decode()
    assert len(out.strip().splitlines()) == 1, out[:2000]
    return json.loads(out)


def test_bench_parse_line():
    line = _bench("--workload", "parse", "--scale", "16", "--edge-factor", "4")
    assert line["verify"] == {"lines": 4 << 16, "equal_to_generated_ids": True}
    assert "equal" in line["cpu_baseline"]["sample"] and line["cpu_baseline"]["value"] > 0
    assert 0 < line["roofline"]["frac"] <= 1 and line["value"] > 0


def test_bench_bip_line():
    line = _bench("--workload", "bip", "--scale", "14", "--edge-factor", "8", "--window-log2", "12")
    v = line["verify"]
    assert v["bipartite"] is True and v["equal_to_cc_counts"] is True and v["vertices"] > 0
    assert line["cpu_baseline"]["value"] > 0 and 0 < line["roofline"]["frac"] <= 1
