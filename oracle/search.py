"""ORACLE (test infrastructure only) — restatement of the reference's transducer search.

Restates, in plain Python/numpy:
  * `core/hotword_context.py:17-184`  ContextGraph (Aho-Corasick; sherpa-onnx context-graph.cc
    semantics): build with max-score shared prefixes (:46-90), BFS fail/output links with
    output-score accumulation (:92-136), non-strict forward_one_step (:138-180), finalize (:182-184)
  * `core/hotword_context.py:191-222` hotword file parsing
  * `core/asr_engine.py:1023-1153` `_ort_beam_search` (modified beam search; greedy is
    beam_size=1): f32 log-softmax, f32 score add (:1099-1100), global
    top-k (:1103-1106), blank/non-blank expansion (:1116-1125), hotword delta after top-k
    (:1127-1131), f64 log-add dedup keyed by the full token sequence (:1133-1138),
    finalize + length-normalised pick (:1142-1153)
  * `core/asr_engine.py:1159-1181` per-token entropy statistics.

This oracle is pinned against the reference itself: tests/golden/make_golden.py drives the
reference's own `_ort_beam_search` with numpy decoder/joiner sessions and commits the
outputs; tests/test_search_oracle.py checks this restatement against them.
"""
from __future__ import annotations

import math
import unicodedata
from collections import deque
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

BLANK = 0
UNK = 2
CTX = 2


class Node:
    __slots__ = ("tok", "tok_score", "node_score", "out_score", "is_end", "kids", "fail", "out")

    def __init__(self, tok=-1, tok_score=0.0, node_score=0.0, out_score=0.0, is_end=False):
        self.tok = tok
        self.tok_score = tok_score
        self.node_score = node_score
        self.out_score = out_score
        self.is_end = is_end
        self.kids: Dict[int, "Node"] = {}
        self.fail: Optional["Node"] = None
        self.out: Optional["Node"] = None


class HotwordGraph:
    def __init__(self, phrases: Sequence[Sequence[int]], scores: Sequence[float]):
        self.root = Node()
        self.root.fail = self.root
        self.nodes: List[Node] = [self.root]
        for seq, sc in zip(phrases, scores):
            if not seq:
                continue
            cur = self.root
            last = len(seq) - 1
            for j, t in enumerate(seq):
                nxt = cur.kids.get(t)
                if nxt is None:
                    ns = cur.node_score + sc
                    nxt = Node(t, sc, ns, ns if j == last else 0.0, j == last)
                    cur.kids[t] = nxt
                    self.nodes.append(nxt)
                else:
                    nxt.tok_score = max(sc, nxt.tok_score)
                    nxt.node_score = cur.node_score + nxt.tok_score
                    if j == last:
                        nxt.is_end = True
                    if nxt.is_end:
                        nxt.out_score = nxt.node_score
                cur = nxt
        self._links()

    def _links(self):
        q = deque()
        for kid in self.root.kids.values():
            kid.fail = self.root
            q.append(kid)
        while q:
            cur = q.popleft()
            for t, kid in cur.kids.items():
                f = cur.fail
                if t in f.kids:
                    f = f.kids[t]
                else:
                    f = f.fail
                    while t not in f.kids:
                        f = f.fail
                        if f.tok == -1:
                            break
                    if t in f.kids:
                        f = f.kids[t]
                kid.fail = f
                o = f
                while not o.is_end:
                    o = o.fail
                    if o.tok == -1:
                        o = None
                        break
                kid.out = o
                if o is not None:
                    kid.out_score += o.out_score
                q.append(kid)

    def step(self, state: Node, t: int) -> Tuple[float, Node]:
        if t in state.kids:
            nd = state.kids[t]
            delta = nd.tok_score
        else:
            nd = state.fail
            while t not in nd.kids:
                nd = nd.fail
                if nd.tok == -1:
                    break
            if t in nd.kids:
                nd = nd.kids[t]
            delta = nd.node_score - state.node_score
        if nd.out_score != 0:
            if nd.is_end:
                matched = nd.node_score
            elif nd.out is not None:
                matched = nd.out.node_score
            else:
                matched = nd.node_score
            return delta + matched - nd.node_score, self.root
        return delta, nd

    @staticmethod
    def finalize(state: Node) -> float:
        return -state.node_score


def parse_hotwords(path: str, default_score: float = 1.5) -> List[Tuple[str, float]]:
    out = []
    with open(path, "r", encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            score = default_score
            if ":" in line:
                head, tail = line.rsplit(":", 1)
                try:
                    score = float(tail.strip())
                    line = head.strip()
                except ValueError:
                    pass
            phrase = unicodedata.normalize("NFC", line.strip().upper())
            if phrase:
                out.append((phrase, score))
    return out


def log_add(a, b):
    """f64 log-add.  Like the reference (core/asr_engine.py:724-728) the non-cutoff branch
    yields an np.float64, which makes the next frame's `lp[i, :] += score` an f64 add
    rounded to f32 (NumPy 2 / NEP 50), while a plain Python float is added in f32."""
    if a < b:
        a, b = b, a
    d = b - a
    return a if d < -36.0 else a + np.log1p(np.exp(d))


def beam_search(enc_out: np.ndarray, decoder: Callable[[np.ndarray], np.ndarray],
                joiner: Callable[[np.ndarray, np.ndarray], np.ndarray], beam: int,
                graph: Optional[HotwordGraph] = None, ties: Optional[list] = None):
    """enc_out float32 (T', D).  Returns (token_ids, frames, tok_logps, T', emit_logits).
    `ties` (checker use): a list that receives every frame whose beam-th and (beam+1)-th
    candidate scores are exactly equal -- there the kept set is whatever np.argpartition's
    introselect leaves (not a stable order), i.e. the reference's result depends on it."""
    Tn = enc_out.shape[0]
    cache: Dict[Tuple[int, int], np.ndarray] = {}

    def dec_rows(ctxs):
        # cache misses go to the decoder as one batch, duplicates included, each hypothesis
        # taking the row of its own batch position and the cache keeping the last one
        # (core/asr_engine.py:1073-1088): row values can depend on the batch shape in BLAS
        rows = [cache.get(c) for c in ctxs]
        miss = [i for i, r in enumerate(rows) if r is None]
        if miss:
            res = decoder(np.array([ctxs[i] for i in miss], dtype=np.int64))
            for j, i in enumerate(miss):
                rows[i] = res[j]
                cache[ctxs[i]] = res[j].copy()
        return np.stack(rows)

    # hyp record: [ys(list), logp(f64), frames, tok_logps, emit_logits, ctx_state]
    hyps: Dict[tuple, list] = {(-1, BLANK): [[-1, BLANK], 0.0, [], [], [],
                                              graph.root if graph else None]}
    for t in range(Tn):
        prev = list(hyps.values())
        H = len(prev)
        ctxs = [tuple(max(0, y) for y in h[0][-CTX:]) for h in prev]
        dec = dec_rows(ctxs)
        enc = np.repeat(enc_out[t:t + 1], H, axis=0)
        logits = joiner(enc, dec).astype(np.float32)
        m = logits.max(axis=-1, keepdims=True)
        sh = logits - m
        lp = sh - np.log(np.exp(sh).sum(axis=-1, keepdims=True))
        for i in range(H):
            lp[i, :] += prev[i][1]  # f32 array += python float (NEP 50: f32 add)
        flat = lp.reshape(-1)
        V = lp.shape[1]
        k = min(beam, flat.shape[0])
        top = np.argpartition(flat, -k)[-k:]
        top = top[np.argsort(flat[top])[::-1]]
        if ties is not None and flat.shape[0] > k:
            kth = flat[top[-1]]
            if np.count_nonzero(flat == kth) > np.count_nonzero(flat[top] == kth):
                ties.append(t)
        nxt: Dict[tuple, list] = {}
        for idx in top:
            hi, tok = int(idx // V), int(idx % V)
            score = float(flat[idx])
            ys, plp, fr, tl, el, cs = prev[hi]
            if tok == BLANK:
                rec = [list(ys), score, list(fr), list(tl), list(el), cs]
            else:
                ncs = cs
                if graph is not None and cs is not None and tok != UNK:
                    dlt, ncs = graph.step(cs, tok)
                    score += dlt
                rec = [ys + [tok], score, fr + [t], tl + [float(lp[hi, tok]) - plp],
                       el + [logits[hi].copy()], ncs]
            key = tuple(rec[0])
            if key in nxt:
                nxt[key][1] = log_add(nxt[key][1], score)
            else:
                nxt[key] = rec
        hyps = nxt
    if graph is not None:
        for rec in hyps.values():
            if rec[5] is not None:
                rec[1] += graph.finalize(rec[5])
    best = max(hyps.values(), key=lambda r: r[1] / max(len(r[0]), 1))
    toks = [y for y in best[0][CTX:] if y > 0]
    return toks, best[2], best[3], Tn, best[4]


def token_entropy(raw_logits: np.ndarray, V: int) -> dict:
    """Per-token statistics over one joiner row (f32 numpy arithmetic as the reference)."""
    max_ent = math.log(V) if V > 1 else 1.0
    a = 1.0 / 3.0
    ts_max = (1.0 / (a - 1.0)) * (1.0 - V ** (1.0 - a)) if V > 1 else 1.0
    z = raw_logits - np.max(raw_logits)
    p = np.exp(z)
    p /= np.sum(p)
    ent = -float(np.sum(p * np.log(p + 1e-30)))
    ts = float((1.0 / (a - 1.0)) * (1.0 - np.sum(p ** a)))
    srt = np.sort(p)[::-1]
    top1 = float(srt[0])
    top2 = float(srt[1]) if len(srt) > 1 else 1e-10
    return {"tsallis_norm": round(float(ts / ts_max if ts_max > 0 else 0.0), 4),
            "margin": round(top1 - top2, 4),
            "entropy_norm": round(ent / max_ent, 4),
            "top1_prob": top1}


def raw_token_stats(raw_logits: np.ndarray) -> Tuple[float, float, float, float]:
    """Unrounded (entropy, sum p^(1/3), top1, top2) in f32 numpy, for kernel comparisons."""
    z = raw_logits - np.max(raw_logits)
    p = np.exp(z)
    p /= np.sum(p)
    ent = -float(np.sum(p * np.log(p + 1e-30)))
    s3 = float(np.sum(p ** (1.0 / 3.0)))
    srt = np.sort(p)[::-1]
    return ent, s3, float(srt[0]), float(srt[1]) if len(srt) > 1 else 1e-10
