"""The sherpa-onnx stream-shaped surface (zasr.offline over the zasr_*stream* C ABI) on an
MI355X: the reference's core/audio_analyzer.py:345-361 call sequence (create_stream ->
accept_waveform -> decode_stream -> stream.result.text / .ys_log_probs) and
streaming_asr.py:224-243's from_transducer(**kwargs) on a reference-layout model directory
give decode_chunk's tokens and log-probs; decode_streams is one batch equal to the single
decodes; the C JSON result agrees with the Python result."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _speech(sec, seed):
    from zasr.synth_audio import synth_speech
    return synth_speech(sec, seed)


@pytest.fixture(scope="module")
def onnx_dir(tmp_path_factory):
    if not gpu_available():
        pytest.skip("no GPU")
    from model_fixtures import tiny_model
    from write_onnx import write_model_dir
    from zasr.model import synth_tokens
    cfg, w, _ = tiny_model(3)
    d = str(tmp_path_factory.mktemp("stream_model") / "model")
    write_model_dir(d, w, synth_tokens(cfg.vocab_size))
    return cfg, d


def _kwargs(d, method="modified_beam_search", beam=8):
    # streaming_asr.py:224-233, verbatim keys
    return {"tokens": os.path.join(d, "tokens.txt"),
            "encoder": glob.glob(os.path.join(d, "encoder*.onnx"))[0],
            "decoder": glob.glob(os.path.join(d, "decoder*.onnx"))[0],
            "joiner": glob.glob(os.path.join(d, "joiner*.onnx"))[0],
            "num_threads": 1, "sample_rate": 16000, "feature_dim": 80,
            "decoding_method": method, "max_active_paths": beam}


@pytest.mark.parametrize("method,beam", [("modified_beam_search", 8), ("greedy_search", 1)])
def test_audio_analyzer_sequence_equals_decode_chunk(onnx_dir, method, beam):
    from zasr import asr_engine as ae
    from zasr.offline import OfflineRecognizer
    cfg, d = onnx_dir
    recognizer = OfflineRecognizer.from_transducer(**_kwargs(d, method, beam), precision="fp32")
    audio = _speech(6.0, 4242)
    # core/audio_analyzer.py:345-361
    stream = recognizer.create_stream()
    stream.accept_waveform(16000, audio.astype(np.float32))
    recognizer.decode_stream(stream)
    result = stream.result
    text = result.text.strip()
    # decode_chunk's search on the same audio (the tuple its word dicts come from)
    rec = ae.create_recognizer(d, max_active_paths=beam, hotwords=([], []), precision="fp32")
    r = rec["handle"].decode([audio], beam=beam)[0]
    assert result.token_ids == r.token_ids.tolist()
    assert result.ys_log_probs == r.log_probs.tolist()
    assert len(result.ys_log_probs) == len(result.tokens) > 0
    id2 = ae._load_tokens(os.path.join(d, "tokens.txt"))
    assert text == "".join(id2[t] for t in result.token_ids).replace("▁", " ").strip()
    conf = float(np.exp(np.mean(result.ys_log_probs)))
    assert 0.0 < conf <= 1.0
    js = json.loads(stream.as_json_string())
    assert js["text"] == result.text and js["tokens"] == result.tokens
    assert js["ys_log_probs"] == result.ys_log_probs
    assert js["timestamps"] == [round(t, 2) for t in result.timestamps]
    ae.clear_model_cache()


def test_decode_streams_is_one_batch_equal_to_single_decodes(onnx_dir):
    from zasr.offline import OfflineRecognizer
    _, d = onnx_dir
    recognizer = OfflineRecognizer.from_transducer(**_kwargs(d), precision="fp32")
    audios = [_speech(s, 900 + i) for i, s in enumerate((3.0, 7.5, 1.2, 0.05))]
    single = []
    for a in audios:
        s = recognizer.create_stream()
        s.accept_waveform(16000, a)
        recognizer.decode_stream(s)
        single.append(s.result)
    streams = []
    for a in audios:
        s = recognizer.create_stream()
        h = len(a) // 3  # accept_waveform appends
        s.accept_waveform(16000, a[:h])
        s.accept_waveform(16000, a[h:])
        streams.append(s)
    recognizer.decode_streams(streams)
    for s, ref in zip(streams, single):
        assert s.result.token_ids == ref.token_ids
        assert s.result.ys_log_probs == ref.ys_log_probs
        assert s.result.timestamps == ref.timestamps
    assert single[-1].token_ids == [] and single[-1].text == ""  # 0.05 s: under 9 frames


def test_stream_errors(onnx_dir):
    from zasr.binding import ZasrError
    from zasr.offline import OfflineRecognizer
    _, d = onnx_dir
    recognizer = OfflineRecognizer.from_transducer(**_kwargs(d), precision="bf16")
    s = recognizer.create_stream()
    with pytest.raises(ZasrError):
        s.accept_waveform(8000, np.zeros(100, np.float32))
    assert s.result.text == ""  # not decoded yet: an empty result
    with pytest.raises(ZasrError):
        s.as_json_string()
    other = OfflineRecognizer.from_transducer(**_kwargs(d), precision="bf16")
    with pytest.raises(ZasrError):
        other.decode_stream(s)  # a stream of another recognizer
    with pytest.raises(FileNotFoundError):
        kw = _kwargs(d)
        kw["encoder"] = os.path.join(d, "missing-encoder.onnx")
        OfflineRecognizer.from_transducer(**kw)


def test_json_result_uses_the_given_symbol_table(onnx_dir, tmp_path):
    """the JSON result reads the tokens file the recognizer was given (sherpa-onnx
    OfflineModelConfig.tokens), not model_dir/tokens.txt."""
    from zasr.offline import OfflineRecognizer
    _, d = onnx_dir
    other = tmp_path / "renamed_tokens.txt"
    with open(os.path.join(d, "tokens.txt"), encoding="utf-8") as f:
        rows = [ln.split() for ln in f if ln.strip()]
    with open(other, "w", encoding="utf-8") as f:
        f.write("".join(f"{'X' + s if int(i) > 2 else s} {i}\n" for s, i in rows))
    kw = _kwargs(d)
    kw["tokens"] = str(other)
    recognizer = OfflineRecognizer.from_transducer(**kw, precision="fp32")
    s = recognizer.create_stream()
    s.accept_waveform(16000, _speech(6.0, 4243))
    recognizer.decode_stream(s)
    js = json.loads(s.as_json_string())
    assert s.result.tokens and all(t.startswith("X") for t in s.result.tokens)
    assert js["tokens"] == s.result.tokens and js["text"] == s.result.text
