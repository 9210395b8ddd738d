"""ViBERT-capu punctuation / capitalisation around the GPU session (BASELINE config 5's
punctuation leg): the host logic of the reference's `GecBERTModel` (core/gec_model.py) and
`PunctuationRestorer.restore` (core/punctuation_restorer_improved.py), restated so that the
transcript text that comes out is the reference's, with the BERT forward on MI355X
(`zasr.binding.VibertSession`, the onnxruntime `run(None, feeds)` surface).

  split_chunks            core/gec_model.py:279-306   56-word chunks, 16-word overlap
  merge_chunks / apply_chunk_merging :308-364   SequenceMatcher over the overlap
  predict / _convert      :366-412, :483-556   mini-batches of 32, softmax, +confidence on
                                     $KEEP, pause-hint nudges, argmax
  get_token_action        :414-443   only $APPEND_<punct> and $TRANSFORM_CASE_* are allowed
  preprocess              :445-481   [$START] + words[:max_len] -> word pieces, input_offsets
  update_final_batch      :558-575   only chunks whose text changed are predicted again
  postprocess_batch       :577-607   edits per chunk (skipped when every label is 0 or the
                                     error probability is below min_error_probability)
  handle_batch            :609-663   up to 3 iterations, chunk merge, punctuation spacing
  get_target_sent_by_edits core/gec_utils.py:31-67 (+ convert_using_case :85-99)
  restore / _post_process core/punctuation_restorer_improved.py:50-133

The word-piece tokenizer is a callable `tokenize(word) -> [piece ids]` (load_word_pieces:
the HF tokenizer of the model dir's vocab.txt, as the reference's _get_indexer builds it),
and `start_id` is the id of the added $START token.  Pinned by tests/golden/punct_cases.json,
made by running the reference's own GecBERTModel / ImprovedPunctuationRestorer on the same
sessions and tokenizer (tests/golden/make_golden_punct.py).
"""
from __future__ import annotations

import re
from difflib import SequenceMatcher
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

START_TOKEN = "$START"
# vocabulary/labels.txt and d_tags.txt of the reference (the model's label namespaces, in
# index order)
LABELS = ["$KEEP", "$TRANSFORM_CASE_CAPITAL", "$APPEND_,", "$APPEND_.", "$TRANSFORM_VERB_VB_VBN",
          "$TRANSFORM_CASE_UPPER", "$APPEND_:", "$APPEND_?", "$TRANSFORM_VERB_VB_VBC",
          "$TRANSFORM_CASE_LOWER", "$TRANSFORM_CASE_CAPITAL_1", "$TRANSFORM_CASE_UPPER_-1",
          "$MERGE_SPACE", "@@UNKNOWN@@", "@@PADDING@@"]
D_TAGS = ["CORRECT", "INCORRECT", "@@UNKNOWN@@", "@@PADDING@@"]
PUNC = (':', ".", ",", "?")


def _softmax(x, axis=-1):
    e = np.exp(x - np.max(x, axis=axis, keepdims=True))
    return e / e.sum(axis=axis, keepdims=True)


def _convert_case(token: str, action: str) -> str:
    """core/gec_utils.py:86-101."""
    if action.endswith("LOWER"):
        return token.lower()
    if action.endswith("UPPER"):
        return token.upper()
    if action.endswith("CAPITAL"):
        return token.capitalize()
    if action.endswith("CAPITAL_1"):
        return token[0] + token[1:].capitalize()
    if action.endswith("UPPER_-1"):
        return token[:-1].upper() + token[-1]
    return token


def target_by_edits(source: List[str], edits) -> List[str]:
    """core/gec_utils.py:32-65 for the edits get_token_action lets through (appended
    punctuation, case transforms); merges never occur, so replace_merge_transforms is the
    identity."""
    target = source[:]
    shift = 0
    for start, end, label, _ in edits:
        pos = start + shift
        if start < 0:
            continue
        src = target[pos] if len(target) > pos else ""
        if label == "":
            del target[pos]
            shift -= 1
        elif start == end:
            word = label.replace("$APPEND_", "")
            if (pos < len(target) and target[pos] == word) or (pos > 0 and target[pos - 1] == word):
                continue
            target[pos:pos] = [word]
            shift += 1
        elif label.startswith("$TRANSFORM_"):
            target[pos] = _convert_case(src, label) if label.startswith("$TRANSFORM_CASE") else src
        elif start == end - 1:
            target[pos] = label.replace("$REPLACE_", "")
    return target


class GecPunctuator:
    """The reference's GecBERTModel configured as PunctuationRestorer builds it
    (split_chunk=True, chunk_size=56, overlap_size=16, max_len=80, iterations=3,
    confidence=0.3; core/punctuation_restorer_improved.py:35-47), one model."""

    def __init__(self, session, tokenize: Callable[[str], Sequence[int]], start_id: int,
                 iterations: int = 3, max_len: int = 80, min_len: int = 3, chunk_size: int = 56,
                 overlap_size: int = 16, min_words_cut: int = 6, confidence: float = 0.3,
                 case_confidence: float = 0.0, min_error_probability: float = 0.0,
                 mini_batch_size: int = 32, pad_id: int = 0):
        self.session = session
        self.tokenize = tokenize
        self.start_id, self.pad_id = int(start_id), int(pad_id)
        self.iterations, self.max_len, self.min_len = iterations, max_len, min_len
        self.chunk_size, self.overlap_size = chunk_size, overlap_size
        self.min_words_cut = min_words_cut
        self.stride = chunk_size - overlap_size
        self.confidence, self.case_confidence = confidence, case_confidence
        self.min_error_probability = min_error_probability
        self.mini_batch_size = mini_batch_size
        self.noop_index = LABELS.index("$KEEP")
        self.incorr_index = D_TAGS.index("INCORRECT")
        self.case_indices = [i for i, t in enumerate(LABELS) if t.startswith("$TRANSFORM_CASE_")]
        self.append_period_index = LABELS.index("$APPEND_.")
        self.append_comma_index = LABELS.index("$APPEND_,")
        self.punc_str = '[' + ''.join(f'\\{x}' for x in PUNC) + ']'
        self.runs = 0           # session.run calls (mini-batches)
        self.rows_run = []      # chunks predicted per iteration
        self.run_shapes = []    # (rows, pieces, word slots) of every session.run

    # ---- chunking (:279-364) ----
    def split_chunks(self, batch, pause_hints=None):
        result, indices = [], []
        hints_result = [] if pause_hints is not None else None
        for b, tokens in enumerate(batch):
            start = len(result)
            n = len(tokens)
            hints = pause_hints[b] if pause_hints is not None else None
            if n <= self.chunk_size:
                result.append(tokens)
                if hints is not None:
                    hints_result.append(hints[:n])
            elif n < self.chunk_size * 2 - self.overlap_size:
                cut = (n + self.overlap_size + 1) // 2
                result += [tokens[:cut], tokens[cut - self.overlap_size:]]
                if hints is not None:
                    hints_result += [hints[:cut], hints[cut - self.overlap_size:]]
            else:
                for i in range(0, n - self.overlap_size, self.stride):
                    result.append(tokens[i:i + self.chunk_size])
                    if hints is not None:
                        hints_result.append(hints[i:i + self.chunk_size])
            indices.append((start, len(result)))
        return result, indices, hints_result

    def _merge_pair(self, tokens, nxt):
        if not tokens:
            return nxt
        src_idx, tgt_idx, src, tgt = [], [], [], []
        num_keep = self.overlap_size - self.min_words_cut
        i = 0
        while len(src_idx) < self.overlap_size and -i < len(tokens):
            i -= 1
            if tokens[i] not in PUNC:
                src_idx.insert(0, i)
                src.insert(0, tokens[i].lower())
        i = 0
        while len(tgt_idx) < self.overlap_size and i < len(nxt):
            if nxt[i] not in PUNC:
                tgt_idx.append(i)
                tgt.append(nxt[i].lower())
            i += 1
        for tag, i1, i2, j1, j2 in SequenceMatcher(None, src, tgt).get_opcodes():
            if tag == "equal":
                if i1 >= num_keep:
                    tail, head = src_idx[i1], tgt_idx[j1]
                    break
                if i2 > num_keep:
                    tail, head = src_idx[num_keep], tgt_idx[j2 - i2 + num_keep]
                    break
            elif tag == "delete" and i1 == 0:
                num_keep += i2 // 2
        return tokens[:tail] + nxt[head:]  # unbound tail / head raise like the reference

    def merge_chunks(self, batch) -> str:
        result: List[str] = []
        if len(batch) == 1 or self.overlap_size == 0:
            for sub in batch:
                result.extend(sub)
        else:
            for sub in batch:
                try:
                    result = self._merge_pair(result, sub)
                except Exception as e:  # the reference prints and keeps what it has (:361)
                    print(e)
        return " ".join(result)

    # ---- model (:475-594) ----
    def preprocess(self, token_batch) -> Optional[Dict[str, np.ndarray]]:
        """[$START] + words[:max_len] through the word-piece tokenizer, right-padded with
        `pad_id`; input_offsets = 0 plus every position whose word id differs from the
        previous position's (word_ids() is None on padding, so a padded row also lists its
        first padding position; a word with no pieces lists nothing), zero-padded."""
        lens = [len(s) for s in token_batch if s]
        if not lens:
            return None
        max_len = min(max(lens), self.max_len)
        rows, wids = [], []
        for seq in token_batch:
            ids, wid = [self.start_id], [0]
            for k, w in enumerate(list(seq)[:max_len]):
                p = list(self.tokenize(w))
                ids += p
                wid += [k + 1] * len(p)
            rows.append(ids)
            wids.append(wid)
        T = max(len(r) for r in rows)
        offs = []
        for wid in wids:
            wid = wid + [None] * (T - len(wid))
            offs.append([0] + [j for j in range(1, T) if wid[j] != wid[j - 1]])
        W = max(len(o) for o in offs)
        B = len(rows)
        feeds = {"input_ids": np.full((B, T), self.pad_id, np.int64),
                 "attention_mask": np.zeros((B, T), np.int64),
                 "token_type_ids": np.zeros((B, T), np.int64),
                 "input_offsets": np.zeros((B, W), np.int64)}
        for i, (r, o) in enumerate(zip(rows, offs)):
            feeds["input_ids"][i, :len(r)] = r
            feeds["attention_mask"][i, :len(r)] = 1
            feeds["input_offsets"][i, :len(o)] = o
        return feeds

    def predict(self, feeds, pause_hints_batch=None):
        n = feeds["input_ids"].shape[0]
        mb = int(self.mini_batch_size or 32)
        if n > mb:
            lg, dt = [], []
            for i in range(0, n, mb):
                a, b = self.session.run(None, {k: v[i:i + mb] for k, v in feeds.items()})
                self.run_shapes.append((a.shape[0],) + feeds["input_ids"].shape[1:] + (a.shape[1],))
                lg.append(a)
                dt.append(b)
                self.runs += 1
            logits, detect = np.concatenate(lg, axis=0), np.concatenate(dt, axis=0)
        else:
            logits, detect = self.session.run(None, feeds)
            self.run_shapes.append((n, feeds["input_ids"].shape[1], logits.shape[1]))
            self.runs += 1
        probs = np.zeros_like(logits, dtype=np.float32)
        err = np.zeros(logits.shape[:1], dtype=np.float32)
        probs += (1 / 1) * _softmax(logits, axis=-1)
        err += (1 / 1) * _softmax(detect, axis=-1)[:, :, self.incorr_index].max(axis=-1)
        if self.confidence != 0.0:
            probs[:, :, self.noop_index] += self.confidence
        if self.case_confidence != 0.0:
            for idx in self.case_indices:
                probs[:, :, idx] += self.case_confidence
        if pause_hints_batch is not None:
            for b, hints in enumerate(pause_hints_batch):
                if hints is None:
                    continue
                for w, gap in enumerate(hints):
                    t = w + 1
                    if t >= probs.shape[1]:
                        break
                    keep = int(probs[b, t].argmax()) == self.noop_index
                    if gap >= 1.0:
                        if keep:
                            probs[b, t, self.noop_index] -= 0.2
                            probs[b, t, self.append_period_index] += 0.2
                    elif gap >= 0.2:
                        if keep:
                            probs[b, t, self.append_comma_index] += 0.2
                    elif gap < 0.1:
                        probs[b, t, self.append_comma_index] -= 0.3
        return probs.max(axis=-1).tolist(), probs.argmax(axis=-1).tolist(), err.tolist()

    def _action(self, index, prob, sugg):
        if prob < self.min_error_probability or sugg in ("@@UNKNOWN@@", "@@PADDING@@", "$KEEP"):
            return None
        if sugg == "$DELETE" or sugg.startswith("$REPLACE_"):
            return None
        if sugg.startswith("$APPEND_"):
            if sugg.replace("$APPEND_", "") not in PUNC:
                return None
            s = e = index + 1
        elif sugg.startswith("$TRANSFORM_CASE_"):
            s, e = index, index + 1
        else:
            return None
        clear = sugg[:] if sugg.startswith("$TRANSFORM_") else sugg[sugg.index("_") + 1:]
        return s - 1, e - 1, clear, prob

    def postprocess_batch(self, batch, probs, idxs, err):
        out = []
        for tokens, p, ix, e in zip(batch, probs, idxs, err):
            length = min(len(tokens), self.max_len)
            if max(ix) == 0 or e < self.min_error_probability:
                out.append(tokens)
                continue
            edits = []
            for i in range(length + 1):
                if ix[i] == self.noop_index:
                    continue
                a = self._action(i, p[i], LABELS[ix[i]])
                if a:
                    edits.append(a)
            out.append(target_by_edits(tokens, edits))
        return out

    @staticmethod
    def update_final_batch(final, pred_ids, pred_batch, prev):
        new_ids = []
        for i, oid in enumerate(pred_ids):
            orig, pred = final[oid], pred_batch[i]
            if orig != pred and pred not in prev[oid]:
                final[oid] = pred
                new_ids.append(oid)
                prev[oid].append(pred)
            elif orig != pred:
                final[oid] = pred
        return final, new_ids

    def handle_batch(self, full_batch, merge_punc=True, pause_hints=None) -> List[str]:
        full_batch, indices, hints = self.split_chunks(full_batch, pause_hints)
        final = full_batch[:]
        prev = {i: [final[i]] for i in range(len(final))}
        short = {i for i in range(len(full_batch)) if len(full_batch[i]) < self.min_len}
        pred_ids = [i for i in range(len(full_batch)) if i not in short]
        for it in range(self.iterations):
            orig = [final[i] for i in pred_ids]
            cur_hints = [hints[i] for i in pred_ids] if (it == 0 and hints is not None) else None
            feeds = self.preprocess(orig)
            if feeds is None:
                break
            self.rows_run.append(len(orig))
            probs, idxs, err = self.predict(feeds, cur_hints)
            final, pred_ids = self.update_final_batch(final, pred_ids,
                                                      self.postprocess_batch(orig, probs, idxs, err),
                                                      prev)
            if not pred_ids:
                break
        out = [self.merge_chunks(final[s:e]) for s, e in indices]
        if merge_punc:
            out = [re.sub(r'\s+(%s)' % self.punc_str, r'\1', x) for x in out]
        return out

    def restore(self, text: str, pause_hints=None) -> str:
        """PunctuationRestorer.restore (core/punctuation_restorer_improved.py:50-78): the whole
        text as one sequence, then the restorer's post-processing."""
        if not text or not text.strip():
            return ""
        try:
            res = self.handle_batch([text.split()],
                                    pause_hints=[pause_hints] if pause_hints is not None else None)
            return post_process(res[0])
        except Exception as e:  # the reference logs and returns the input text (:75-78)
            import logging
            logging.getLogger("zasr.punct").error("restore failed: %s", e, exc_info=True)
            return text


def load_word_pieces(model_dir: str, lowercase: bool = False):
    """The word-piece tokenizer of a ViBERT model dir as GecBERTModel._get_indexer builds it
    (core/gec_model.py:220-235: AutoTokenizer from the dir's vocab.txt, do_basic_tokenize
    False, $START added as the last id).  Returns (tokenize(word) -> piece ids, start_id,
    pad_id); tokenize is memoised per word, and with is_split_into_words each word is
    tokenized on its own, so per-word pieces concatenate to the batch encoding."""
    from functools import lru_cache

    from transformers import AutoTokenizer
    tok = AutoTokenizer.from_pretrained(model_dir, do_basic_tokenize=False,
                                        do_lower_case=lowercase, model_max_length=1024)
    tok.add_tokens([START_TOKEN])
    start_id = len(tok) - 1

    @lru_cache(maxsize=1 << 18)
    def pieces(word: str) -> Tuple[int, ...]:
        return tuple(tok([word], is_split_into_words=True, add_special_tokens=False)["input_ids"])

    return pieces, start_id, int(tok.pad_token_id or 0)


def post_process(text: str) -> str:
    """core/punctuation_restorer_improved.py:80-134."""
    text = text.replace(':', ' ')
    text = re.sub(r',+', ',', text)
    text = re.sub(r'\.{4,}', '...', text)
    text = re.sub(r',\s*\.', '.', text)
    out = []
    for sent in re.split(r'(?<=[.!?])\s+', text):
        if len(sent.split()) < 8 and sent.count(',') > 1:
            parts = sent.split(',', 1)
            if len(parts) > 1:
                k = parts[1].find(',')
                if k != -1:
                    parts[1] = parts[1][:k] + parts[1][k + 1:].replace(',', '')
                sent = parts[0] + ',' + parts[1]
        out.append(sent)
    text = ' '.join(out)
    text = re.sub(r'([,.!?])([^\s])', r'\1 \2', text)
    text = re.sub(r'\s+([,.!?])', r'\1', text)
    text = re.sub(r'^,\s*', '', text)
    text = re.sub(r'\.\s*,', '. ', text)
    text = re.sub(r'\s+', ' ', text)
    text = re.sub(r'(^|[.!?]\s+)([^\W_])', lambda m: m.group(1) + m.group(2).upper(), text)
    return text.strip()
