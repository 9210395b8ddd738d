"""zasr.punct (the GecBERTModel / ImprovedPunctuationRestorer host logic around the ViBERT
session) against tests/golden/punct_cases.json -- the reference's own handle_batch and
restore run on the same sessions and tokenizer (tests/golden/make_golden_punct.py): the
output text and the digest of every session run (the mini-batched feeds of each iteration,
i.e. which chunks are re-run) are equal."""
import json
import os

import numpy as np
import pytest

from punct_sessions import Recorder, ScriptedSession, write_model_dir

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "punct_cases.json"), encoding="utf-8"))


@pytest.fixture(scope="module")
def pieces(tmp_path_factory):
    from zasr.punct import load_word_pieces
    return load_word_pieces(write_model_dir(str(tmp_path_factory.mktemp("vib"))))


def oracle_session(seed):
    from oracle.vibert import VibertOracle
    from zasr.vibert import synth_weights, vibert_tiny
    cfg = vibert_tiny()
    w = synth_weights(cfg, seed)
    w["classifier.weight"] = w["classifier.weight"] * np.float32(40.0)
    o = VibertOracle(cfg, w)

    class S:
        def run(self, names, feeds):
            return o.run(feeds["input_ids"], feeds["attention_mask"], feeds["token_type_ids"],
                         feeds["input_offsets"])
    return S()


def run_case(c, session, pieces):
    from zasr.punct import GecPunctuator
    tok, start_id, pad_id = pieces
    rec = Recorder(session)
    g = GecPunctuator(rec, tok, start_id, pad_id=pad_id)
    if c["kind"] == "restore":
        out = g.restore(c["text"], pause_hints=c["pause_hints"])
    else:
        out = g.handle_batch([t.split() for t in c["texts"]], pause_hints=c["pause_hints"])
    return out, rec.calls, g


def _spec(c):
    s = c["session"]
    return ScriptedSession(s["seed"], s["scale"], s["keep_bias"]) if s["kind"] == "scripted" else None


@pytest.mark.parametrize("i", [i for i, c in enumerate(CASES) if c["session"]["kind"] == "scripted"])
def test_scripted_cases_equal_reference(i, pieces):
    c = CASES[i]
    out, calls, _ = run_case(c, _spec(c), pieces)
    assert calls == c["calls"]
    assert out == c["out"]


@pytest.mark.parametrize("i", [i for i, c in enumerate(CASES) if c["session"]["kind"] == "oracle"])
def test_oracle_vibert_cases_equal_reference(i, pieces):
    c = CASES[i]
    out, calls, _ = run_case(c, oracle_session(c["session"]["seed"]), pieces)
    assert calls == c["calls"]
    assert out == c["out"]


def test_fixtures_cover_the_paths():
    """The fixtures exercise: mini-batches (>32 chunks in one iteration), re-running only the
    changed chunks (a later iteration with fewer rows), pause hints, chunk merging, edits of
    every allowed kind (appended . , ? : and case transforms)."""
    runs = [len(c["calls"]) for c in CASES]
    assert max(runs) >= 6
    outs = " ".join(c["out"] if isinstance(c["out"], str) else " ".join(c["out"]) for c in CASES)
    for p in ".,?":
        assert p in outs
    assert any(c["pause_hints"] for c in CASES)
    assert any(w.isupper() and len(w) > 1 for w in outs.split())


def test_rerun_only_changed_chunks(pieces):
    c = next(c for c in CASES if c["kind"] == "batch" and c["session"]["kind"] == "scripted")
    _, _, g = run_case(c, _spec(c), pieces)
    assert g.rows_run[0] > 32 and g.rows_run[-1] < g.rows_run[0]


def test_post_process_rules():
    from zasr.punct import post_process
    # ':' -> ' ', ',,' -> ',', ', .' -> '.', one comma in a short sentence is kept
    assert post_process("xin chào: tôi ,, là , . bạn") == "Xin chào tôi, là. Bạn"
    # short sentence with 3 commas keeps the first and drops the rest; leading ', ' dropped
    assert post_process(", a, b, c d. e") == "A b c d. E"
    assert post_process("x.y ,z ; w?  q") == "X. Y, z ; w? Q"
    assert post_process("") == ""


def test_preprocess_word_ids_offsets(pieces):
    """[$START] first, the first piece of every word, the first padding position of a padded
    row (its word id is None), zero-padded offsets -- the feeds the reference builds with
    batch.word_ids() (core/gec_model.py:445-481)."""
    from zasr.punct import GecPunctuator
    tok, start_id, pad_id = pieces
    g = GecPunctuator(None, tok, start_id, pad_id=pad_id)
    f = g.preprocess([["xin", "chàoxyz", "bạn"], ["tôi"]])
    p = [list(tok(w)) for w in ("xin", "chàoxyz", "bạn")]
    assert f["input_ids"][0].tolist() == [start_id] + sum(p, [])
    assert f["input_offsets"][0].tolist() == [0, 1, 1 + len(p[0]), 1 + len(p[0]) + len(p[1])]
    n1 = 1 + len(tok("tôi"))
    assert f["input_offsets"][1, :3].tolist() == [0, 1, n1]
    assert f["attention_mask"][1].sum() == n1
