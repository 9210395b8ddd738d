"""Host logic of the full pipe (zasr.pipeline): the word chunking of the punctuation model
(core/gec_model.py:279-305 split_chunks), the ONNX feeds of GecBERTModel.preprocess
(:445-481) with the synthetic word pieces, the edit loop and the transcript handed to the
restorer.  The reference's own handle_batch / restore pin the whole punctuation logic in
tests/test_punct.py."""
import numpy as np

from zasr.pipeline import (l2_normalise, make_punctuator, split_word_chunks,
                           transcript_for_punctuation, vibert_feeds, word_pieces)


def _w(n):
    return [f"w{i}" for i in range(n)]


def test_split_word_chunks_cases():
    assert split_word_chunks(_w(0)) == [[]]
    assert split_word_chunks(_w(56)) == [_w(56)]
    # 57 <= n < 96: two halves sharing 16 words, cut at (n + 17) // 2
    c = split_word_chunks(_w(57))
    assert c == [_w(57)[:37], _w(57)[21:]]
    c = split_word_chunks(_w(95))
    assert [len(x) for x in c] == [56, 55] and c[0][-16:] == c[1][:16]
    # n >= 96: windows of 56 every 40 while start < n - 16
    c = split_word_chunks(_w(96))
    assert [x[0] for x in c] == ["w0", "w40"] and [len(x) for x in c] == [56, 56]
    c = split_word_chunks(_w(200))
    assert [x[0] for x in c] == ["w0", "w40", "w80", "w120", "w160"]
    assert [len(x) for x in c] == [56, 56, 56, 56, 40]
    # chunk 48 / overlap 12 (GecBERTModel's defaults, :64-65)
    c = split_word_chunks(_w(100), 48, 12)
    assert [x[0] for x in c] == ["w0", "w36", "w72"]


def test_vibert_feeds_offsets_and_padding():
    V = 1000
    f = vibert_feeds([["a", "b", "c"], ["d"]], V)
    ids, off, am = f["input_ids"], f["input_offsets"], f["attention_mask"]
    assert ids[0, 0] == V - 1 and ids[1, 0] == V - 1          # START token first
    pa = [word_pieces(w, V) for w in "abc"]
    n0 = 1 + sum(len(p) for p in pa)
    assert ids.shape[1] == n0 and am[0].sum() == n0
    assert off[0, :4].tolist() == [0, 1, 1 + len(pa[0]), 1 + len(pa[0]) + len(pa[1])]
    # the padded row gets the first padding position as an extra offset (word id None)
    n1 = 1 + len(word_pieces("d", V))
    assert off[1, :3].tolist() == [0, 1, n1] and am[1].sum() == n1
    assert (f["token_type_ids"] == 0).all()
    assert all(5 <= i <= V - 2 for w in "abcd" for i in word_pieces(w, V))


def test_punctuator_applies_edits_and_stops_when_stable():
    """A session that always predicts $APPEND_. (label 3) at every slot: iteration 1 appends a
    period after every word and one at the $START slot (before the first word, as the
    reference does); iteration 2 predicts the same edits, which target_by_edits skips (a
    period is already adjacent), so no chunk changes and the loop ends after 2 runs."""
    calls = []

    class Sess:
        def run(self, names, feeds):
            B, W = feeds["input_offsets"].shape
            calls.append(B)
            lg = np.zeros((B, W, 15), np.float32)
            lg[:, :, 3] = 10.0
            return [lg, np.zeros((B, W, 4), np.float32)]

    g = make_punctuator(Sess(), 1000, mini_batch=32)
    out = g.handle_batch([_w(20)])[0]
    assert out == ". " + " ".join(w + "." for w in _w(20))
    assert g.rows_run == [1, 1]


def test_transcript_for_punctuation():
    ws = [{"text": "xin", "start": 0.0, "end": 0.3}, {"text": "ờ", "start": 0.4, "end": 0.5},
          {"text": "chào", "start": 0.9, "end": 1.2}, {"text": "BẠN", "start": 1.25, "end": 1.5}]
    text, hints = transcript_for_punctuation(ws)
    assert text == "Xin chào bạn"      # filler dropped, str.capitalize lowers the rest
    assert hints == [0.6000000000000001, 0.050000000000000044, 1.0]
    assert transcript_for_punctuation(ws[:1]) == ("Xin", None)


def test_l2_normalise():
    e = np.array([[3.0, 4.0], [0.0, 0.0]], np.float32)
    assert np.allclose(l2_normalise(e), [[0.6, 0.8], [0.0, 0.0]])
