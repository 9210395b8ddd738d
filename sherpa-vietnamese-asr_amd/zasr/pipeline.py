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
engine's stream.  Host work: word post-processing, the merge, the word chunking and the
synthetic word-piece ids (the ViBERT vocab.txt tokenizer is absent: every word maps to 1-2
ids by a stable hash, the START token is the last id as after special_tokens_fix).
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
    while the start is before n - overlap."""
    n = len(words)
    if n <= chunk_size:
        return [list(words)]
    if n < chunk_size * 2 - overlap_size:
        cut = (n + overlap_size + 1) // 2
        return [list(words[:cut]), list(words[cut - overlap_size:])]
    stride = chunk_size - overlap_size
    return [list(words[i:i + chunk_size]) for i in range(0, n - overlap_size, stride)]


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


def vibert_feeds(batch: Sequence[Sequence[str]], vocab_size: int, max_len: int = MAX_LEN
                 ) -> Dict[str, np.ndarray]:
    """GecBERTModel.preprocess (core/gec_model.py:475-517): [START] + words[:max_len], word
    pieces padded to the batch's longest, input_offsets = every position whose word id
    differs from the previous one's -- the first piece of every word, plus the first padding
    position of a padded row (its word id is None), zero-padded to the longest list."""
    start_id = vocab_size - 1
    L = min(max(len(s) for s in batch), max_len)
    rows, offs = [], []
    for seq in batch:
        ids, off = [start_id], [0]
        for w in list(seq)[:L]:
            off.append(len(ids))
            ids += _pieces(w, vocab_size)
        rows.append(ids)
        offs.append(off)
    T = max(len(r) for r in rows)
    for r, o in zip(rows, offs):
        if len(r) < T:
            o.append(len(r))
    W = max(len(o) for o in offs)
    B = len(rows)
    input_ids = np.zeros((B, T), np.int64)
    mask = np.zeros((B, T), np.int64)
    offsets = np.zeros((B, W), np.int64)
    for i, (r, o) in enumerate(zip(rows, offs)):
        input_ids[i, :len(r)] = r
        mask[i, :len(r)] = 1
        offsets[i, :len(o)] = o
    return {"input_ids": input_ids, "attention_mask": mask,
            "token_type_ids": np.zeros((B, T), np.int64), "input_offsets": offsets}


def punctuate(session, words: Sequence[str], vocab_size: int, iterations: int = ITERATIONS,
              mini_batch: int = MINI_BATCH) -> Tuple[List[np.ndarray], int]:
    """ViBERT passes over the transcript's word chunks: `iterations` passes of every chunk of
    at least 3 words (core/gec_model.py:623-654; the reference re-runs only chunks whose text
    changed, so this is its upper bound), mini-batches of `mini_batch` rows (32 in the
    reference; <= 0: the whole pass in one run -- rows are independent and the padding is the
    whole pass's either way, so the logits are the same bits).  Returns the per-chunk label
    argmax of the last pass (softmax is monotone: argmax of the logits, :579-581) and the
    number of session runs."""
    chunks = [c for c in split_word_chunks(list(words)) if len(c) >= 3]
    labels: List[np.ndarray] = [np.zeros(0, np.int64)] * len(chunks)
    runs = 0
    if not chunks:
        return labels, runs
    for _ in range(iterations):
        # the whole batch is preprocessed (padded) at once, then sliced (:636-640, :380-392)
        feeds = vibert_feeds(chunks, vocab_size)
        mb = mini_batch if mini_batch > 0 else len(chunks)
        for b in range(0, len(chunks), mb):
            lg, _ = session.run(None, {k: v[b:b + mb] for k, v in feeds.items()})
            runs += 1
            am = lg.argmax(-1)
            for i in range(am.shape[0]):
                labels[b + i] = am[i, 1:1 + min(len(chunks[b + i]), MAX_LEN)]
    return labels, runs


def l2_normalise(embs: np.ndarray) -> np.ndarray:
    """The reference's per-window normalisation (speaker_diarization_senko_campp_optimized.py:
    607-611): divide by the L2 norm when it exceeds 1e-10."""
    n = np.linalg.norm(embs, axis=1, keepdims=True)
    return np.where(n > 1e-10, embs / np.maximum(n, 1e-30), embs)


class FullPipe:
    """One file through the config-5 pipe on one GPU (module docstring).  The audio goes to
    HBM once; `run()` returns the merged word dicts, the punctuation label ids per word chunk,
    the L2-normalised window embeddings and their (region, first frame, frames) plan.

    rec: zasr.binding.Recognizer; recd: {"id2token", "vocab_size"} of its tokens; emb:
    CamppEmbedder; vib: VibertSession (ONNX session surface); vib_vocab: ViBERT vocabulary
    size incl. START."""

    def __init__(self, rec, recd, emb, vib, vib_vocab: int, beam: int = 1,
                 campp_batch: int = 4096, iterations: int = ITERATIONS, vib_batch: int = 0):
        self.rec, self.recd, self.emb, self.vib = rec, recd, emb, vib
        self.vib_vocab, self.beam, self.B, self.iterations = vib_vocab, beam, campp_batch, iterations
        self.vib_batch = vib_batch  # <= 0: one ViBERT run per pass (punctuate)

    def prepare(self, audio: np.ndarray) -> None:
        import torch
        from zasr.plan import plan_chunks
        a = np.ascontiguousarray(audio, np.float32)
        self.n = a.shape[0]
        plan = plan_chunks(a)                      # decode chunks, 3 s overlap
        regions = plan_chunks(a, overlap_sec=0.0)  # diarization speech regions
        self.c_off = [s for s, _, _ in plan]
        self.c_len = [e - s for s, e, _ in plan]
        self.r_off = [s for s, _, _ in regions]
        self.r_len = [e - s for s, e, _ in regions]
        # window count bound: (frames - 150) / 60 + 2 per region
        self.cap = sum(max(1, (n // 160) // 60 + 2) for n in self.r_len)
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
        return self.rec.decode_device_batches(self.d_audio.data_ptr(), self.c_off * passes,
                                              self.c_len * passes, [n] * passes,
                                              beam=self.beam, stream=stream)

    def words(self, res) -> Tuple[List[Dict], int]:
        from zasr.asr_engine import result_words
        from zasr.merge import merge_chunks_with_overlap
        chunks = [{"words": result_words(self.recd, r, n, s / 16000.0),
                   "audio_start_abs": s / 16000.0, "audio_end_abs": (s + n) / 16000.0}
                  for r, s, n in zip(res, self.c_off, self.c_len)]
        words, _ = merge_chunks_with_overlap(chunks)
        return words, sum(int(r.token_ids.size) for r in res)

    def decode_words(self, stream: int) -> Tuple[List[Dict], int]:
        return self.words(self.decode(stream))

    def embed_windows(self, stream: int):
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
                    labels, runs = punctuate(self.vib, [w["text"] for w in words],
                                             self.vib_vocab, self.iterations, self.vib_batch)
                    # the copy runs on (and waits for) the CAM++ stream only, never on `main`
                    # where the next decode is in flight
                    with torch.cuda.stream(self.s_campp):
                        embs = l2_normalise(self.d_emb[:len(reg)].cpu().numpy())
                    outs.append({"words": words, "tokens": tokens, "labels": labels,
                                 "vibert_runs": runs, "embeddings": embs,
                                 "windows": np.stack([reg, first, nfr], 1)})
        return outs
