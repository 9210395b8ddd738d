"""Localise a beam-search divergence between the HIP search and the oracle search on the SAME
encoder output (development tool; test infrastructure, imports oracle/).

Rebuilds tests/test_gpu_e2e.py's widened case (the first WIDE_CHUNKS planner chunks of the
bench weights, hotword.txt + emitted n-grams), runs, for the chunks given on the command line,
the HIP search on the oracle's encoder output and the oracle search, with and without the
hotword graph and with hotword.txt only, and reports the first differing token / frame and
the oracle's top hypotheses around that frame.  Writes gpurun_out/beam_divergence.json.

    python sherpa-vietnamese-asr_amd/tools/beam_divergence.py 3 13
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"),
          os.path.join(ROOT, "sherpa-vietnamese-asr_amd")):
    sys.path.insert(0, p)


def traced_beam(enc_out, decoder, joiner, beam, graph, t_lo, t_hi):
    """oracle.search.beam_search with the kept hypotheses (tokens, score) recorded for
    frames t_lo..t_hi (a copy of its loop; the result must equal beam_search's)."""
    from oracle.search import BLANK, CTX, UNK, log_add
    Tn = enc_out.shape[0]
    cache = {}
    trace = {}

    def dec_rows(ctxs):
        rows = [cache.get(c) for c in ctxs]
        miss = [i for i, r in enumerate(rows) if r is None]
        if miss:
            res = decoder(np.array([ctxs[i] for i in miss], dtype=np.int64))
            for j, i in enumerate(miss):
                rows[i] = res[j]
                cache[ctxs[i]] = res[j].copy()
        return np.stack(rows)

    hyps = {(-1, BLANK): [[-1, BLANK], 0.0, graph.root if graph else None]}
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
            lp[i, :] += prev[i][1]
        flat = lp.reshape(-1)
        V = lp.shape[1]
        k = min(beam, flat.shape[0])
        top = np.argpartition(flat, -k)[-k:]
        top = top[np.argsort(flat[top])[::-1]]
        if t_lo <= t <= t_hi:
            srt = np.sort(flat)[::-1]
            trace[t] = {"kth": float(srt[k - 1]), "k+1th": float(srt[k]) if len(srt) > k else None,
                        "gap_k": float(srt[k - 1] - srt[k]) if len(srt) > k else None}
        nxt = {}
        for idx in top:
            hi, tok = int(idx // V), int(idx % V)
            score = float(flat[idx])
            ys, plp, cs = prev[hi]
            if tok == BLANK:
                rec = [list(ys), score, cs]
            else:
                ncs = cs
                if graph is not None and cs is not None and tok != UNK:
                    dlt, ncs = graph.step(cs, tok)
                    score += dlt
                rec = [ys + [tok], score, ncs]
            key = tuple(rec[0])
            if key in nxt:
                nxt[key][1] = log_add(nxt[key][1], score)
            else:
                nxt[key] = rec
        hyps = nxt
        if t_lo <= t <= t_hi:
            trace[t]["hyps"] = sorted([(round(r[1], 5), r[0][-4:]) for r in hyps.values()],
                                      reverse=True)
    return trace


def main():
    import bench
    from model_fixtures import m_model
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search, parse_hotwords
    from oracle.zipformer import ZipformerOracle
    from synth_case import hotword_token_ids, ngram_phrases
    from test_gpu_e2e import HOTWORDS, WIDE_CHUNKS, edit_distance
    from zasr.binding import Recognizer

    which = [int(a) for a in sys.argv[1:]] or [3]
    cfg, w, path = m_model(bench.WEIGHT_SEED)
    orc = ZipformerOracle(cfg, w)
    chunks = bench.make_chunks(WIDE_CHUNKS * 36.0 + 40.0, bench.AUDIO_SEED)[:WIDE_CHUNKS]
    enc0 = orc.encoder(fbank(chunks[0]))
    g0 = beam_search(enc0, orc.decoder, orc.joiner, 1)
    seqs, scores = hotword_token_ids(parse_hotwords(HOTWORDS), cfg.vocab_size)
    ng = ngram_phrases(g0[0])
    graphs = {"none": ([], []), "hotword_txt": (seqs, scores),
              "hotword_txt+ngrams": (seqs + ng, scores + [2.0] * len(ng))}
    out = {}
    for i in which:
        enc = orc.encoder(fbank(chunks[i]))
        for gname, (ph, sc) in graphs.items():
            graph = HotwordGraph(ph, sc) if ph else None
            ref = beam_search(enc, orc.decoder, orc.joiner, 8, graph)
            kw = {"hotwords": ph, "hotword_scores": sc} if ph else {}
            rec = Recognizer(path, "modified_beam_search", 8, precision="fp32", **kw)
            r = rec.search([enc], beam=8)[0]
            rec.close()
            got = r.token_ids.tolist()
            entry = {"equal": got == ref[0], "edit_distance": edit_distance(got, ref[0]),
                     "n_ref": len(ref[0]), "n_got": len(got)}
            if got != ref[0]:
                d = next((j for j, (a, b) in enumerate(zip(got, ref[0])) if a != b),
                         min(len(got), len(ref[0])))
                fr_ref = ref[1][d] if d < len(ref[1]) else None
                fr_got = int(r.frames[d]) if d < len(r.frames) else None
                entry.update({"first_diff_token": d, "frame_ref": fr_ref, "frame_got": fr_got,
                              "ref_tokens": ref[0][max(0, d - 3):d + 4],
                              "got_tokens": got[max(0, d - 3):d + 4],
                              "ref_frames": ref[1][max(0, d - 3):d + 4],
                              "got_frames": r.frames[max(0, d - 3):d + 4].tolist(),
                              "got_log_probs": r.log_probs[max(0, d - 3):d + 4].tolist(),
                              "ref_log_probs": ref[2][max(0, d - 3):d + 4]})
                t0 = min(x for x in (fr_ref, fr_got) if x is not None)
                entry["oracle_trace"] = {str(k): v for k, v in traced_beam(
                    enc, orc.decoder, orc.joiner, 8, graph, max(0, t0 - 3), t0 + 1).items()}
            out[f"chunk{i}/{gname}"] = entry
            print(f"chunk {i} {gname}: {json.dumps({k: v for k, v in entry.items() if k != 'oracle_trace'})}",
                  flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "beam_divergence.json"), "w") as f:
        json.dump(out, f, indent=1, default=float)


if __name__ == "__main__":
    main()
