"""Host-side rows of SURVEY §8a: chunk planning (K) and the ROVER block vote (L), against
fixtures produced by the reference's own functions (tests/golden/make_golden_host.py)."""
import copy
import json
import os

import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def plans():
    return _load("plan_cases.json")


def test_planner_matches_reference(plans):
    from make_golden_host import audio_sum, plan_audio
    from zasr.plan import plan_chunks, silent_regions
    for c in plans["cases"]:
        a = plan_audio(c["seed"], c["seconds"])
        assert audio_sum(a) == c["audio_sha"], "synthetic audio drifted; regenerate fixtures"
        assert [list(r) for r in silent_regions(a)] == c["silent_regions"]
        assert [list(p) for p in plan_chunks(a)] == c["plan"]


def test_long_segment_split_matches_reference(plans):
    from zasr.plan import split_long_segment
    for c in plans["long_segments"]:
        assert [list(x) for x in split_long_segment(c["start"], c["end"])] == c["chunks"]


def test_concat_time_map_matches_reference(plans):
    from zasr.plan import concat_to_original
    m = plans["concat_map"]
    omap = [tuple(x) for x in m["offset_map"]]
    got = [concat_to_original(t, omap) for t in m["times"]]
    assert got == pytest.approx(m["original"], abs=1e-12)


def test_vad_gap_merge_and_concat():
    import numpy as np
    from zasr.plan import concat_speech, merge_vad_gaps
    segs = [(0, 100), (150, 300), (300 + 5 * 16000 + 1, 400000)]
    assert merge_vad_gaps(segs) == [(0, 300), (300 + 5 * 16000 + 1, 400000)]
    a = np.arange(1000, dtype=np.float32)
    c, omap = concat_speech(a, [(10, 20), (100, 105)])
    assert c.tolist() == list(range(10, 20)) + list(range(100, 105))
    assert omap == [(0, 10, 10), (10, 100, 5)]


def test_rover_merge_matches_reference():
    from zasr.rover import rover_merge
    g = _load("rover_cases.json")
    phrases = g["hotword_phrases"]
    for k, c in enumerate(g["cases"]):
        merged, dis = rover_merge(copy.deepcopy(c["A"]), copy.deepcopy(c["B"]), phrases)
        assert sorted(dis) == c["disagree"], k
        assert merged == c["merged"], k
