"""Chunk-overlap merge (zasr.merge) vs fixtures from the reference's own
merge_chunks_with_overlap / find_overlap_alignment (core/asr_engine.py:70-237;
tests/golden/make_golden_merge.py)."""
import copy
import json
import os

import pytest

from zasr.merge import align_overlap, fuzzy_equal, merge_chunks_with_overlap, overlap_key

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merge_cases.json"),
                       encoding="utf-8"))


@pytest.mark.parametrize("i", range(len(CASES)), ids=[f"{c['mode']}{i}" for i, c in enumerate(CASES)])
def test_merge_matches_reference(i):
    c = CASES[i]
    chunks = copy.deepcopy(c["chunks"])
    where = {id(w): [k, j] for k, ch in enumerate(chunks) for j, w in enumerate(ch["words"])}
    words, text = merge_chunks_with_overlap(chunks)
    assert [where[id(w)] for w in words] == c["picked"]
    assert text == c["text"]


def test_fixture_modes_cover_every_action():
    acts = set()
    for c in CASES:
        ch = c["chunks"]
        for k in range(1, len(ch)):
            prev = ch[k - 1]
            tail = [w for w in prev["words"]
                    if w["local_start"] >= max(0, prev["audio_end_abs"] - prev["audio_start_abs"] - 3.0)]
            head = [w for w in ch[k]["words"] if w["local_start"] < 3.0]
            acts.add(align_overlap(tail, head)[1])
    assert {"none", "cut_head", "drop_head", "drop_tail"} <= acts, acts


def test_word_keys():
    assert overlap_key(" Xin, ") == "xin"
    assert not fuzzy_equal("chào", "chao")  # difflib ratio 0.75 < 0.8, 4 chars neither containing the other
    assert fuzzy_equal("thanhs", "thanh")     # containment
    assert fuzzy_equal("thành", "thành")
    assert fuzzy_equal("nguyen", "nguyenx")  # substring, both longer than 2
    assert not fuzzy_equal("", "a")
