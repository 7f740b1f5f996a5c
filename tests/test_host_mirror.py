"""CPU: host-side logic of the operator mirror (windowing, tree schedule) — no device calls."""
import json
import os

import numpy as np
import pytest

from gsgpu.aggregation import SimpleEdgeStream
from gloo_tree import tree_schedule

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_event_time_windows_match_example():
    k = json.load(open(os.path.join(GOLD, "reference_kats.json")))["ConnectedComponentsExample"]
    s = SimpleEdgeStream(k["src"], k["dst"], k["timestamps"])
    wins = s.windows(k["merge_window_ms"], None)
    assert [[w.start, w.stop] for w in wins] == [w["edges"] for w in k["event_time_windows"]]
    assert len(wins) == 11


def test_count_windows():
    s = SimpleEdgeStream(np.arange(10), np.arange(10))
    assert [(w.start, w.stop) for w in s.windows(1000, 4)] == [(0, 4), (4, 8), (8, 10)]
    assert [(w.start, w.stop) for w in s.windows(1000, None)] == [(0, 10)]
    assert SimpleEdgeStream([], []).windows(5, 3) == []


def test_descending_timestamps_rejected():
    s = SimpleEdgeStream([1, 2], [2, 3], [100, 50])
    with pytest.raises(ValueError):
        s.windows(10, None)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
def test_tree_schedule_reaches_rank0(world):
    # simulate: every rank's data must arrive at rank 0; each rank sends exactly once (rank>0)
    holds = {r: {r} for r in range(world)}
    scheds = {r: tree_schedule(r, world) for r in range(world)}
    rounds = len(scheds[0])
    assert rounds == (0 if world == 1 else int(np.ceil(np.log2(world))))
    done = set()
    for i in range(rounds):
        for r in range(world):
            if r in done:
                continue
            role, peer = scheds[r][i]
            if role == "send":
                assert scheds[peer][i] == ("recv", r)
                holds[peer] |= holds[r]
                done.add(r)
    assert holds[0] == set(range(world))
    assert done == set(range(1, world))
