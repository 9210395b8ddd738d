"""ROVER ensemble of two Zipformer models.

GPU side: one fbank per chunk shared by both models (core/asr_engine.py:2346-2350), both
decodes batched over all chunks (`decode_chunks_rover`).  Host side: the reference's block
vote `rover_merge_words` (core/asr_engine.py:1446-1577), restated as `rover_merge`:

  * the two word sequences are aligned on normalised text (difflib opcodes, no autojunk);
  * equal / delete blocks keep model A's words;
  * a replace block keeps the side with the higher mean word confidence
    (margin_min * (1 - tsallis_max), else prob, :1336-1351), after a hotword bonus of
    0.5 x (fraction of the block's words covered by a hotword phrase found in the block plus
    up to 3 equal-context words on each side) for the only side that has one (:1374-1443);
    ties keep A; chosen words are flagged `_disagree`;
  * B-only words join when their confidence exceeds 0.20, flagged `_disagree`, and are
    dropped again if an A word with the same normalised text starts within 0.15 s;
  * the result is ordered by start time; the set of `_disagree` positions is returned.
"""
from __future__ import annotations

import re
from functools import lru_cache
import unicodedata
from difflib import SequenceMatcher
from typing import Dict, List, Optional, Sequence, Set, Tuple

HOTWORD_BONUS = 0.5
CONTEXT_WORDS = 3
INSERT_MIN_CONF = 0.20
DUP_WINDOW_SEC = 0.15

Word = Dict


_NON_WORD = re.compile(r"[^\w]", flags=re.UNICODE)


@lru_cache(maxsize=1 << 16)
def normalize_word(text: str) -> str:
    """lowercase, NFC, word characters only (core/asr_engine.py:44-49); memoised (a
    transcript repeats its syllables)."""
    return _NON_WORD.sub("", unicodedata.normalize("NFC", text.lower().strip()))


def word_confidence(w: Word) -> float:
    m, ts = w.get("margin_min"), w.get("tsallis_max")
    if m is not None and ts is not None:
        return m * (1.0 - ts)
    return w.get("prob", 0.5)


def block_confidence(ws: Sequence[Word]) -> float:
    return sum(word_confidence(w) for w in ws) / len(ws) if ws else 0.0


def hotword_ratio(block: Sequence[Word], before: Optional[Sequence[Word]],
                  after: Optional[Sequence[Word]], phrases: Sequence[str]) -> float:
    """Fraction of `block`'s words that lie (at least partly) inside an occurrence of a
    hotword phrase in the text of before + block + after (phrases lower-cased, longest first)."""
    if not block or not phrases:
        return 0.0
    seq = list(before or []) + list(block) + list(after or [])
    norms = [normalize_word(w["text"]) for w in seq]
    text = " ".join(norms)
    covered = bytearray(len(text))
    for ph in phrases:
        i = text.find(ph)
        while i >= 0:
            covered[i:i + len(ph)] = b"\x01" * len(ph)
            i = text.find(ph, i + 1)
    if not any(covered):
        return 0.0
    first = len(before or [])
    hits, pos = 0, 0
    for k, nw in enumerate(norms):
        at = text.find(nw, pos)
        if at < 0:
            continue
        if first <= k < first + len(block) and any(covered[at:at + len(nw)]):
            hits += 1
        pos = at + len(nw)
    return hits / len(block)


def rover_merge(words_a: List[Word], words_b: List[Word],
                hotword_phrases: Sequence[str] = ()) -> Tuple[List[Word], Set[int]]:
    """Block vote between model A (primary) and model B words of one chunk.  Mutates the
    chosen word dicts' `_disagree` flag like the reference; returns (merged, disagree)."""
    if not words_a:
        return (list(words_b) if words_b else []), set()
    if not words_b:
        return list(words_a), set()
    phrases = sorted((p.lower() for p in hotword_phrases), key=len, reverse=True)
    ops = SequenceMatcher(None, [normalize_word(w["text"]) for w in words_a],
                          [normalize_word(w["text"]) for w in words_b],
                          autojunk=False).get_opcodes()
    out: List[Word] = []
    supplements: List[int] = []  # ids of B words added by insert blocks
    for k, (tag, i1, i2, j1, j2) in enumerate(ops):
        if tag in ("equal", "delete"):
            out.extend(words_a[i1:i2])
        elif tag == "insert":
            for w in words_b[j1:j2]:
                if word_confidence(w) > INSERT_MIN_CONF:
                    w["_disagree"] = True
                    supplements.append(id(w))
                    out.append(w)
        else:  # replace
            blk_a, blk_b = words_a[i1:i2], words_b[j1:j2]
            ctx = [None, None, None, None]  # before a, before b, after a, after b
            if k > 0 and ops[k - 1][0] == "equal":
                _, pi1, pi2, pj1, pj2 = ops[k - 1]
                ctx[0] = words_a[max(pi1, pi2 - CONTEXT_WORDS):pi2]
                ctx[1] = words_b[max(pj1, pj2 - CONTEXT_WORDS):pj2]
            if k + 1 < len(ops) and ops[k + 1][0] == "equal":
                _, ni1, ni2, nj1, nj2 = ops[k + 1]
                ctx[2] = words_a[ni1:min(ni2, ni1 + CONTEXT_WORDS)]
                ctx[3] = words_b[nj1:min(nj2, nj1 + CONTEXT_WORDS)]
            ca, cb = block_confidence(blk_a), block_confidence(blk_b)
            ha = hotword_ratio(blk_a, ctx[0], ctx[2], phrases)
            hb = hotword_ratio(blk_b, ctx[1], ctx[3], phrases)
            if ha > 0 and hb == 0:
                ca += ha * HOTWORD_BONUS
            elif hb > 0 and ha == 0:
                cb += hb * HOTWORD_BONUS
            chosen = blk_b if cb > ca else blk_a
            for w in chosen:
                w["_disagree"] = True
            out.extend(chosen)
    out.sort(key=lambda w: w["start"])
    if supplements:
        sup = set(supplements)
        kept: List[Word] = []
        for w in out:
            if id(w) in sup:
                nw = normalize_word(w["text"])
                if any(id(x) not in sup and abs(x["start"] - w["start"]) < DUP_WINDOW_SEC
                       and normalize_word(x["text"]) == nw for x in kept):
                    continue
            kept.append(w)
        out = kept
    return out, {i for i, w in enumerate(out) if w.get("_disagree")}


def decode_chunks_rover(rec_a, rec_b, chunks, time_offsets, hotword_phrases: Sequence[str] = ()):
    """Both models over the same chunks with one shared fbank per chunk (computed on the GPU
    through model A's handle), then the block vote per chunk.  Returns a list of
    (merged_words, disagree_indices) per chunk."""
    import numpy as np
    from zasr.asr_engine import decode_chunks
    ha = rec_a["handle"]
    feats = [ha.fbank(np.asarray(c, np.float32)) for c in chunks]
    words_a = decode_chunks(rec_a, chunks, time_offsets, precomputed_features=feats)
    words_b = decode_chunks(rec_b, chunks, time_offsets, precomputed_features=feats)
    return [rover_merge(a, b, hotword_phrases) for a, b in zip(words_a, words_b)]


def rover_device_many(rec_a, rec_b, recd_a, recd_b, d_wav: int, offsets, lengths, k: int,
                      beam: int, hotword_phrases: Sequence[str] = (), sub_batches: int = 1,
                      passes_per_call: int = 1, mine: Optional[Sequence[int]] = None,
                      gather: bool = True, tokens_out: Optional[list] = None):
    """k passes of one file's chunk plan (waveforms in HBM) through the ROVER pair on one GPU
    (BASELINE config 4): model A (primary, 30M) and model B (68M) decode every chunk
    (`zasr_decode_device`, each on its own engine streams, concurrently: two worker threads,
    the GIL is released inside the ctypes calls), then the per-chunk block vote and the
    chunk-overlap merge on the host -- while the GPU already decodes the next passes.
    Reference: core/asr_engine.py:2018-2047 (the pair), :2346-2350 (both models per chunk),
    :1446-1577 (vote), :182-237 (merge).  The reference shares one fbank per chunk to save CPU
    time; here each engine computes it on the device from the same audio (bit-identical
    features, ~1 ms per hour).  Each decode call takes `passes_per_call` passes, each pass
    `sub_batches` consecutive batches, through the engine's batch pipeline
    (zasr_decode_device_batches: the next batch's encoder under this batch's search; beam
    search keeps two batches' searches in flight), results identical.  Returns [(merged
    words, disagreements per chunk, tokens of A, tokens of B)] per pass.

    mine: strong scaling over the ranks of an initialised torch.distributed group (one process
    per GPU, BASELINE config 4's "sharded across 8 GPUs"): this rank decodes and votes only
    the chunk indices `mine` (its zasr.shard.lpt_partition share of the SAME plan on every
    rank), the voted chunks are gathered to every rank in chunk order (a host object gather,
    zasr.shard.gather_chunks: the vote is per chunk, so the only exchange is its result) and
    every rank merges the whole file; disagreements / tokens are this rank's.  gather=False
    (bench.py --proxy-ranks, one process standing in for one rank): merge this share alone.
    tokens_out: if a list, each pass appends (A's token ids per chunk, B's token ids per chunk)
    of the chunks this call decoded (bench.py's oracle agreement)."""
    from concurrent.futures import ThreadPoolExecutor

    from zasr.asr_engine import result_words
    from zasr.merge import merge_chunks_with_overlap
    from zasr.shard import gather_chunks
    n_all = len(lengths)
    if mine is not None:
        mine = list(mine)
        offsets, lengths = [offsets[i] for i in mine], [lengths[i] for i in mine]
    offsets, lengths = list(offsets), list(lengths)
    n = len(lengths)
    if n == 0:  # more ranks than chunks: nothing to decode, still part of every gather
        out = []
        for _ in range(k):
            words, _ = merge_chunks_with_overlap(gather_chunks([], n_all))
            out.append((words, [], 0, 0))
        return out
    nb = max(1, min(int(sub_batches), n))
    sizes = [n * (i + 1) // nb - n * i // nb for i in range(nb)]
    g = max(1, int(passes_per_call))

    def dec(h, passes):
        if nb == 1 and passes == 1:
            return h.decode_device(d_wav, offsets, lengths, beam=beam)
        return h.decode_device_batches(d_wav, offsets * passes, lengths * passes, sizes * passes,
                                       beam=beam)

    calls = [min(g, k - i) for i in range(0, k, g)]
    out = []
    with ThreadPoolExecutor(2) as ex:
        fa, fb = ex.submit(dec, rec_a, calls[0]), ex.submit(dec, rec_b, calls[0])
        for ci, passes in enumerate(calls):
            ra_all, rb_all = fa.result(), fb.result()
            if ci + 1 < len(calls):
                fa, fb = ex.submit(dec, rec_a, calls[ci + 1]), ex.submit(dec, rec_b, calls[ci + 1])
            for p in range(passes):
                ra, rb = ra_all[p * n:(p + 1) * n], rb_all[p * n:(p + 1) * n]
                chunks, dis = [], []
                for a, b, off, ln in zip(ra, rb, offsets, lengths):
                    t0 = off / 16000.0
                    merged, d = rover_merge(result_words(recd_a, a, ln, t0),
                                            result_words(recd_b, b, ln, t0), hotword_phrases)
                    chunks.append({"words": merged, "audio_start_abs": t0,
                                   "audio_end_abs": (off + ln) / 16000.0})
                    dis.append(len(d))
                if tokens_out is not None:
                    tokens_out.append(([x.token_ids.tolist() for x in ra],
                                       [x.token_ids.tolist() for x in rb]))
                if mine is not None and gather:
                    chunks = gather_chunks(list(zip(mine, chunks)), n_all)
                words, _ = merge_chunks_with_overlap(chunks)
                out.append((words, dis, sum(int(x.token_ids.size) for x in ra),
                            sum(int(x.token_ids.size) for x in rb)))
    return out
