"""Host-side word post-processing of the drop-in `decode_chunk` vs the reference's own
output (golden fixtures from core/asr_engine.py:1209-1326), on CPU: the search result is
the oracle's (pinned separately) with raw joiner rows, exercising the same BPE merge,
timestamps, probabilities and entropy aggregation code the GPU path uses."""
import glob
import json
import os

import numpy as np
import pytest

from zasr.asr_engine import _words_from_search
from oracle.search import HotwordGraph, beam_search
from synth_case import case_config, dec_joiner_weights, enc_out_for, np_decoder, np_joiner
from zasr.model import synth_tokens

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = [p for p in sorted(glob.glob(os.path.join(GOLD, "search_*.json")))
         if "decode_chunk" in json.load(open(p))]


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_decode_chunk_words_match_reference(path):
    g = json.load(open(path))
    cfg = case_config(g["kind"])
    w = dec_joiner_weights(g["kind"], g["seed"])
    enc = enc_out_for(g["kind"], g["seed"], g["T"], cfg.joiner_dim)
    graph = HotwordGraph(g["phrases"], g["scores"]) if g["hotwords"] else None
    toks, frames, lps, T, emit = beam_search(enc, lambda y: np_decoder(w, y),
                                             lambda e, d: np_joiner(w, e, d), g["beam"], graph)
    id2token = dict(enumerate(synth_tokens(cfg.vocab_size)))
    dc = g["decode_chunk"]
    words = _words_from_search(id2token, cfg.vocab_size, dc["n_samples"], dc["time_offset"],
                               toks, frames, lps, T, emit)
    ref = dc["words"]
    assert len(words) == len(ref)
    for a, b in zip(words, ref):
        assert set(a) == set(b)
        for k, v in b.items():
            if isinstance(v, float):
                assert a[k] == pytest.approx(v, abs=1e-12), k
            else:
                assert a[k] == v, k


def test_dropin_install_rebinds_hot_path_names():
    """zasr.dropin.install on a stand-in module object: hot-path names rebound, the rest
    (pipeline, merges, get_ort) left alone, clear_model_cache wrapped (call-through)."""
    import types
    import zasr.asr_engine as ours
    from zasr.dropin import ENGINE_NAMES, install
    ref = types.ModuleType("core_asr_engine_standin")
    ref.TranscriberPipeline = object
    ref.rover_merge_words = lambda a, b: (a, set())
    sentinel_get_ort = lambda: "ort"
    ref.get_ort = sentinel_get_ort
    calls = []
    ref.clear_model_cache = lambda which="all": calls.append(which)
    for n in ENGINE_NAMES:
        setattr(ref, n, None)
    done = install(ref)
    assert ref.create_recognizer is ours.create_recognizer
    assert ref.decode_chunk is ours.decode_chunk
    assert ref.compute_fbank_ort is ours.compute_fbank_ort
    assert ref.TranscriberPipeline is object
    assert ref.get_ort is sentinel_get_ort
    ref.clear_model_cache("restorer")
    assert calls == ["restorer"]
    assert "asr_engine.decode_chunk" in done
    with pytest.raises(ValueError):
        install(ours)
    ours.set_host_module(None)


def test_dropin_install_vad_is_opt_in():
    import types
    import zasr.asr_engine as ours
    import zasr.vad_utils as ours_vad
    from zasr.dropin import VAD_NAMES, install
    ref = types.ModuleType("core_asr_engine_standin")
    ref.get_vad_segments = ref.unload_vad_model = None
    install(ref)
    assert ref.get_vad_segments is None  # no vad_module: the reference's VAD stays
    vad = types.ModuleType("core_vad_utils_standin")
    vad.BASE_DIR = "/opt/app"
    for n in VAD_NAMES:
        setattr(vad, n, None)
    done = install(ref, vad_module=vad)
    assert ref.get_vad_segments is ours_vad.get_vad_segments
    assert vad._get_vad_session is ours_vad._get_vad_session
    assert "vad_utils.get_vad_segments" in done
    assert ours_vad.model_dir() == "/opt/app/models/silero-vad" or "ZASR_VAD_MODEL_DIR" in os.environ
    with pytest.raises(ValueError):
        install(ref, vad_module=ours_vad)
    ours_vad.set_base_dir(None)
    ours.set_host_module(None)
