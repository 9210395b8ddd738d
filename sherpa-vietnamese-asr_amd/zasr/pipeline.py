"""The full transcription pipe of BASELINE config 5 on one GPU: Zipformer decode of the
planned chunks + CAM++ speaker embeddings of the speech regions + ViBERT-capu punctuation of
the merged transcript.

Reference order (core/asr_engine.py TranscriberPipeline.run): plan chunks (:2115-2161) ->
decode (:2250-2397) -> merge_chunks_with_overlap (:2469-2494, zasr.merge) -> diarization
embeddings of the speech regions (core/speaker_diarization_senko_campp_optimized.py:519-605,
1.5 s windows every 0.6 s, batches, L2-normalised) -> punctuation of the full text
(:2908-2935 -> core/punctuation_restorer_improved.py:35-47: GecBERTModel with split_chunk,
chunk_size 56, overlap 16, max_len 80, 3 iterations; core/gec_model.py:279-305 split_chunks,
:366-412 mini-batches of 32 through the ONNX session, :475-517 preprocess).

On the GPU: the CAM++ front end and embeddings run on their own stream while the decode runs
(they only read the audio); the punctuation model runs after the merge, on the ViBERT
engine's stream.  Host work: word post-processing, the merge, and the reference's
punctuation host logic (zasr.punct: chunking, softmax + confidence + pause nudges, edits,
re-running only the changed chunks, chunk merge, the restorer's post-processing).  Word
pieces come from the model dir's vocab.txt (zasr.punct.load_word_pieces) when it has one;
the synthetic benchmark model has none, so every word maps to 1-2 ids by a stable hash, the
START token being the last id as after special_tokens_fix.
"""
from __future__ import annotations

import hashlib
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

import numpy as np

CHUNK_WORDS = 56      # core/punctuation_restorer_improved.py:39
OVERLAP_WORDS = 16    # :40
MAX_LEN = 80          # :41
ITERATIONS = 3        # :42
MINI_BATCH = 32       # core/gec_model.py:189, 382


def split_word_chunks(words: Sequence[str], chunk_size: int = CHUNK_WORDS,
                      overlap_size: int = OVERLAP_WORDS) -> List[List[str]]:
    """core/gec_model.py:279-305 for one sequence: whole when it fits, two halves sharing
    `overlap_size` words below 2 * chunk - overlap, else chunks every chunk - overlap words
    while the start is before n - overlap (zasr.punct.GecPunctuator.split_chunks)."""
    from zasr.punct import GecPunctuator
    g = GecPunctuator(None, None, 0, chunk_size=chunk_size, overlap_size=overlap_size)
    return [list(c) for c in g.split_chunks([list(words)])[0]]


@lru_cache(maxsize=1 << 18)
def _pieces(word: str, vocab_size: int) -> Tuple[int, ...]:
    h = hashlib.blake2b(word.encode("utf-8"), digest_size=8).digest()
    v = int.from_bytes(h, "little")
    span = vocab_size - 2 - 5
    if (v >> 40) % 8 == 0:
        return (5 + v % span, 5 + (v >> 20) % span)
    return (5 + v % span,)


def word_pieces(word: str, vocab_size: int) -> List[int]:
    """Synthetic word-piece ids of one word (stable hash; ids 5 .. vocab_size - 2, ~1 in 8
    words split in two; memoised per word like a tokenizer's vocabulary lookup)."""
    return list(_pieces(word, vocab_size))


def make_punctuator(session, vocab_size: int, tokenizer=None, mini_batch: int = 0,
                    **kw):
    """zasr.punct.GecPunctuator (the reference's GecBERTModel host logic) over `session`.
    tokenizer: (tokenize, start_id, pad_id) from zasr.punct.load_word_pieces for a model dir
    with its vocab.txt; None -> the synthetic hashed word pieces (START = the last id).
    mini_batch <= 0: one session run per iteration (rows are independent and the padding is
    the iteration's either way, so the logits are the reference's 32-row mini-batches' bits,
    tests/test_gpu_pipe.py)."""
    from zasr.punct import GecPunctuator
    if tokenizer is None:
        tokenizer = (lambda w: _pieces(w, vocab_size), vocab_size - 1, 0)
    tok, start_id, pad_id = tokenizer
    return GecPunctuator(session, tok, start_id, pad_id=pad_id,
                         mini_batch_size=mini_batch if mini_batch > 0 else 1 << 30, **kw)


def vibert_feeds(batch: Sequence[Sequence[str]], vocab_size: int) -> Dict[str, np.ndarray]:
    """GecBERTModel.preprocess (core/gec_model.py:445-481) of `batch` with the synthetic word
    pieces (zasr.punct.GecPunctuator.preprocess)."""
    return make_punctuator(None, vocab_size).preprocess(batch)


FILLER_WORDS = {"à", "ờ", "ừ", "ơ", "uh", "um"}   # core/asr_engine.py:1584


def transcript_for_punctuation(words: Sequence[Dict]) -> Tuple[str, List[float]]:
    """The text and pause hints the reference hands to restorer.restore after the merge
    (core/asr_engine.py): filler words dropped (remove_filler_words :1587-1608), full_text =
    the words joined by spaces, str.capitalize()d (:2577-2580), pause_hints[i] = the gap
    after word i clipped at 0, 1.0 after the last word, None with fewer than 2 words or when
    the count differs from the text's word count (:3118-3132)."""
    ws = [w for w in words if w["text"].lower() not in FILLER_WORDS]
    text = " ".join(w["text"] for w in ws)
    if text:
        text = text.capitalize()
    hints = None
    if len(ws) >= 2:
        hints = [max(0.0, ws[i + 1].get("start", 0) - ws[i].get("end", 0)) for i in range(len(ws) - 1)]
        hints.append(1.0)
        if len(hints) != len(text.split()):
            hints = None
    return text, hints


def l2_normalise(embs: np.ndarray) -> np.ndarray:
    """The reference's per-window normalisation (speaker_diarization_senko_campp_optimized.py:
    607-611): divide by the L2 norm when it exceeds 1e-10."""
    n = np.linalg.norm(embs, axis=1, keepdims=True)
    return np.where(n > 1e-10, embs / np.maximum(n, 1e-30), embs)


class FullPipe:
    """One file through the config-5 pipe on one GPU (module docstring).  The audio goes to
    HBM once; `run()` returns the merged word dicts, the punctuated transcript (the
    reference's restorer output), the L2-normalised window embeddings and their (region,
    first frame, frames) plan.

    rec: zasr.binding.Recognizer; recd: {"id2token", "vocab_size"} of its tokens; emb:
    CamppEmbedder; vib: VibertSession (ONNX session surface); vib_vocab: ViBERT vocabulary
    size incl. START."""

    def __init__(self, rec, recd, emb, vib, vib_vocab: int, beam: int = 1,
                 campp_batch: int = 4096, iterations: int = ITERATIONS, vib_batch: int = 0,
                 tokenizer=None, confidence: float = 0.3, case_confidence: float = 0.0,
                 shard: bool = False):
        """shard: strong scaling over the ranks of an initialised torch.distributed group (one
        process per GPU, every rank given the same file): each rank decodes its
        zasr.shard.lpt_partition share of the chunk plan and embeds its share of the speech
        regions; the per-chunk words are gathered to every rank in chunk order and merged
        there, every rank runs the restorer's host logic on the same transcript with each
        ViBERT run's rows split over the ranks (zasr.shard.RowShardedSession), and the window
        embeddings are gathered in region order.  Without a group it is the one-GPU pipe."""
        from zasr.shard import RowShardedSession
        self.rec, self.recd, self.emb, self.vib = rec, recd, emb, vib
        self.vib_vocab, self.beam, self.B, self.iterations = vib_vocab, beam, campp_batch, iterations
        self.shard = bool(shard)
        # <= 0: one ViBERT run per iteration (make_punctuator)
        self.punct = make_punctuator(RowShardedSession(vib) if self.shard else vib, vib_vocab,
                                     tokenizer, vib_batch, iterations=iterations,
                                     confidence=confidence, case_confidence=case_confidence)

    def punctuate(self, words: Sequence[Dict]) -> Tuple[str, int, List[int]]:
        """restorer.restore of the merged transcript (zasr.punct; the reference's
        ImprovedPunctuationRestorer.restore): edits applied, later iterations re-run only the
        chunks whose text changed.  Returns (text, session runs, rows per iteration)."""
        text, hints = transcript_for_punctuation(words)
        r0, n0 = self.punct.runs, len(self.punct.rows_run)
        out = self.punct.restore(text, pause_hints=hints)
        return out, self.punct.runs - r0, self.punct.rows_run[n0:]

    def prepare(self, audio: np.ndarray) -> None:
        import torch
        from zasr.plan import plan_chunks
        a = np.ascontiguousarray(audio, np.float32)
        self.n = a.shape[0]
        plan = plan_chunks(a)                      # decode chunks, 3 s overlap
        regions = plan_chunks(a, overlap_sec=0.0)  # diarization speech regions
        self.c_off_all = [s for s, _, _ in plan]
        self.c_len_all = [e - s for s, e, _ in plan]
        self.r_off_all = [s for s, _, _ in regions]
        self.r_len_all = [e - s for s, e, _ in regions]
        n_c, n_r = len(plan), len(regions)
        self.mine_c, self.mine_r = list(range(n_c)), list(range(n_r))
        if self.shard:
            from zasr.shard import _dist, lpt_partition
            dist = _dist()
            if dist is not None:
                world, rank = dist.get_world_size(), dist.get_rank()
                self.mine_c = lpt_partition(self.c_len_all, world)[rank]
                self.mine_r = lpt_partition(self.r_len_all, world)[rank]
        # this rank's chunks and regions (all of them on one GPU)
        self.c_off = [self.c_off_all[i] for i in self.mine_c]
        self.c_len = [self.c_len_all[i] for i in self.mine_c]
        self.r_off = [self.r_off_all[i] for i in self.mine_r]
        self.r_len = [self.r_len_all[i] for i in self.mine_r]
        # window count bound: (frames - 150) / 60 + 2 per region
        self.cap = max(1, sum(max(1, (n // 160) // 60 + 2) for n in self.r_len))
        self.d_audio = torch.from_numpy(a).cuda()
        self.d_feats = torch.empty((self.cap, 150, 80), dtype=torch.float32, device="cuda")
        self.d_emb = torch.empty((self.cap, self.emb.dim), dtype=torch.float32, device="cuda")
        self.s_campp = torch.cuda.Stream()
        # the audio upload above ran on the current stream: complete it here, so the CAM++
        # stream (which reads only the audio) never has to wait on the decode stream
        torch.cuda.synchronize()

    def decode(self, stream: int, passes: int = 1):
        """Results of `passes` decodes of the file's chunks (one call: consecutive batches
        through the engine's batch pipeline when passes > 1), chunk order, pass after pass."""
        if passes == 1:
            return self.rec.decode_device(self.d_audio.data_ptr(), self.c_off, self.c_len,
                                          beam=self.beam, stream=stream)
        n = len(self.c_len)
        if n == 0:  # more ranks than chunks
            return []
        return self.rec.decode_device_batches(self.d_audio.data_ptr(), self.c_off * passes,
                                              self.c_len * passes, [n] * passes,
                                              beam=self.beam, stream=stream)

    def words(self, res) -> Tuple[List[Dict], int]:
        from zasr.asr_engine import result_words
        from zasr.merge import merge_chunks_with_overlap
        chunks = [{"words": result_words(self.recd, r, n, s / 16000.0),
                   "audio_start_abs": s / 16000.0, "audio_end_abs": (s + n) / 16000.0}
                  for r, s, n in zip(res, self.c_off, self.c_len)]
        if self.shard:
            from zasr.shard import gather_chunks
            chunks = gather_chunks(list(zip(self.mine_c, chunks)), len(self.c_len_all))
        words, _ = merge_chunks_with_overlap(chunks)
        return words, sum(int(r.token_ids.size) for r in res)

    def decode_words(self, stream: int) -> Tuple[List[Dict], int]:
        return self.words(self.decode(stream))

    def embed_windows(self, stream: int):
        if not self.r_len:
            z = np.zeros(0, np.int32)
            return z, z, z
        reg, first, nfr = self.emb.windows_device(self.d_audio.data_ptr(), self.r_off, self.r_len,
                                                  self.d_feats.data_ptr(), self.cap, stream=stream)
        W, D = len(reg), self.emb.dim
        for b in range(0, W, self.B):
            self.emb.embed_device(self.d_feats.data_ptr() + b * 150 * 80 * 4, min(self.B, W - b),
                                  150, self.d_emb.data_ptr() + b * D * 4, stream)
        return reg, first, nfr

    def run(self) -> Dict:
        return self.run_many(1)[0]

    def run_many(self, k: int, passes_per_call: int = 1) -> List[Dict]:
        """k passes of the file through the pipe (k files of a job, here the same audio),
        pipelined: the decode of the next passes (a ctypes call on a worker thread: the GIL is
        released while the GPU decodes; `passes_per_call` passes per call share the engine's
        batch pipeline) runs while this thread post-processes a pass's words, merges them and
        runs its punctuation; CAM++ runs on its own stream beside both."""
        import torch
        from concurrent.futures import ThreadPoolExecutor
        main = torch.cuda.current_stream()
        n = len(self.c_len)
        g = max(1, int(passes_per_call))
        calls = [min(g, k - i) for i in range(0, k, g)]
        outs: List[Dict] = []
        with ThreadPoolExecutor(1) as ex:
            fut = ex.submit(self.decode, main.cuda_stream, calls[0])
            for ci, passes in enumerate(calls):
                res_all = fut.result()
                if ci + 1 < len(calls):
                    fut = ex.submit(self.decode, main.cuda_stream, calls[ci + 1])
                for p in range(passes):
                    # CAM++ on its own stream: it reads only the (already uploaded) audio, so
                    # it is not ordered behind the next passes' decode queued on `main`
                    reg, first, nfr = self.embed_windows(self.s_campp.cuda_stream)
                    words, tokens = self.words(res_all[p * n:(p + 1) * n])
                    text, runs, rows = self.punctuate(words)
                    # the copy runs on (and waits for) the CAM++ stream only, never on `main`
                    # where the next decode is in flight
                    with torch.cuda.stream(self.s_campp):
                        embs = l2_normalise(self.d_emb[:len(reg)].cpu().numpy())
                    win = np.stack([np.asarray(self.mine_r, np.int64)[np.asarray(reg, np.int64)]
                                    if len(reg) else np.zeros(0, np.int64), first, nfr], 1)
                    if self.shard:
                        embs, win = self._gather_windows(embs, win)
                    outs.append({"words": words, "tokens": tokens, "text": text,
                                 "vibert_runs": runs, "vibert_rows": rows, "embeddings": embs,
                                 "windows": win,
                                 "token_ids": [r.token_ids.tolist()
                                               for r in res_all[p * n:(p + 1) * n]]})
        return outs

    def _gather_windows(self, embs: np.ndarray, win: np.ndarray):
        """Every rank's window embeddings and (region, first frame, frames) rows, in region
        order (regions are whole per rank, windows in order within a region)."""
        from zasr.shard import gather_chunks
        part = []
        for ri in self.mine_r:
            sel = win[:, 0] == ri
            part.append((ri, (embs[sel], win[sel])))
        got = gather_chunks(part, len(self.r_len_all))
        dim = embs.shape[1] if embs.ndim == 2 else self.emb.dim
        e = [g[0] for g in got if len(g[0])]
        w = [g[1] for g in got if len(g[1])]
        return (np.concatenate(e) if e else np.zeros((0, dim), np.float32),
                np.concatenate(w) if w else np.zeros((0, 3), np.int64))
