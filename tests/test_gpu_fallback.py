"""The f16x3 mode's fp16 operand range: an activation beyond 65504 makes the f16x3
encoder output non-finite; the engine detects it, drains its streams and reports it, and the
public decode path (zasr.binding.Recognizer, hence create_recognizer / decode_chunk /
OfflineRecognizer) re-decodes with a bf16x6 engine of the same model, returning what a bf16x6
recognizer returns -- where the fp32 reference would have produced a transcript, the drop-in
does too.

The out-of-range model: the tiny Zipformer with encoder_embed.conv.0 scaled to |w| <= 3e4 (the
weights stay below 65504, so the load-time check passes), so the first convolution's outputs (~1e5-1e6)
overflow fp16 as the next convolution's split operand; f32-range modes stay finite.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hot_model(tmp_path_factory):
    if not gpu_available():
        pytest.skip("no GPU")
    from zasr.model import save_model_dir, synth_tokens, synth_weights, zipformer_tiny
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, 5)
    k = np.float32(3e4 / np.abs(w["encoder_embed.conv.0.weight"]).max())
    w["encoder_embed.conv.0.weight"] = w["encoder_embed.conv.0.weight"] * k
    w["encoder_embed.conv.0.bias"] = w["encoder_embed.conv.0.bias"] * k
    assert np.abs(w["encoder_embed.conv.0.weight"]).max() < 65504
    d = str(tmp_path_factory.mktemp("hot"))
    save_model_dir(d, cfg, w, synth_tokens(cfg.vocab_size))
    return d


@pytest.mark.parametrize("method,beam", [("greedy_search", 1), ("modified_beam_search", 4)])
def test_f16x3_out_of_range_falls_back_to_bf16x6(hot_model, method, beam):
    from zasr.binding import Recognizer
    from zasr.synth_audio import synth_speech
    audio = [synth_speech(6.0, 71), synth_speech(3.5, 72)]
    ref = Recognizer(hot_model, method, beam, precision="bf16x6")
    want = ref.decode(audio)
    ref.close()
    assert all(np.all(np.isfinite(r.log_probs)) for r in want)
    rec = Recognizer(hot_model, method, beam, precision="f16x3")
    try:
        got = rec.decode(audio)
        assert rec._fallback is not None, "the f16x3 engine did not report the range overflow"
        # the engine is still usable after the drained error: a second call decodes again
        got2 = rec.decode(audio)
    finally:
        rec.close()
    for a, b, c in zip(got, want, got2):
        assert a.token_ids.tolist() == b.token_ids.tolist() == c.token_ids.tolist()
        assert a.T == b.T
        np.testing.assert_array_equal(a.log_probs, b.log_probs)


@pytest.mark.parametrize("method,beam", [("greedy_search", 1), ("modified_beam_search", 4)])
def test_offline_stream_out_of_range_falls_back_to_bf16x6(hot_model, method, beam):
    """The sherpa-onnx stream surface (core/audio_analyzer.py:345-361, streaming_asr.py:358):
    OfflineRecognizer at its f16x3 default decodes through zasr_decode_stream(s), not through
    Recognizer.decode, so it carries the same fallback -- decode_stream and decode_streams
    re-decode on a bf16x6 engine, and result / as_json_string read the re-decoded streams."""
    import json
    import os
    from zasr.binding import Recognizer
    from zasr.offline import OfflineRecognizer
    from zasr.synth_audio import synth_speech
    audio = [synth_speech(6.0, 81), synth_speech(3.5, 82), synth_speech(2.0, 83)]
    ref = Recognizer(hot_model, method, beam, precision="bf16x6")
    wres = ref.decode(audio)
    ref.close()
    want = [r.token_ids.tolist() for r in wres]
    rec = OfflineRecognizer(hot_model, os.path.join(hot_model, "tokens.txt"),
                            decoding_method=method, max_active_paths=beam, precision="f16x3")
    ss = [rec.create_stream() for _ in audio]
    for s, a in zip(ss, audio):
        s.accept_waveform(16000, a[: len(a) // 2])
        s.accept_waveform(16000, a[len(a) // 2:])
    rec.decode_streams(ss[:2])
    rec.decode_stream(ss[2])
    assert rec._fallback is not None, "the f16x3 engine did not report the range overflow"
    for s, w, r in zip(ss, want, wres):
        assert s.result.num_frames == r.T > 0
        assert s.result.token_ids == w
        assert s.result.text == "".join(rec._syms.get(t, "") for t in w)
        assert json.loads(s.as_json_string())["text"] == s.result.text
