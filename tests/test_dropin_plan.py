"""Plan-ahead routing of the drop-in decode_chunk on CPU (no GPU): the reference's two-worker
loop (core/asr_engine.py:2326-2397) calls decode_chunk once per chunk; after the planner's
find_silent_regions call registered the plan (zasr.dropin wraps it), the whole plan must be
decoded in ONE batched call per recognizer handle, and every chunk's words must equal what the
per-chunk path returns.  The handle is a deterministic stand-in whose result depends only on a
chunk's samples (the real engine's batched == per-chunk property is tested on the GPU,
tests/test_gpu_dropin.py)."""
import threading
from types import SimpleNamespace

import numpy as np

from zasr import asr_engine as ae
from zasr.plan import best_split, plan_chunks, silent_regions
from zasr.synth_audio import synth_speech


class FakeHandle:
    """decode(chunks) -> one result per chunk computed from the chunk's own samples."""

    def __init__(self):
        self.calls = []
        self.lock = threading.Lock()

    def _one(self, a):
        a = np.asarray(a, np.float32)
        n = max(1, a.shape[0] // 4000)
        toks = (np.abs(a[::4000][:n]) * 1e4).astype(np.int64) % 60 + 3
        return SimpleNamespace(token_ids=toks, frames=np.arange(n, dtype=np.int64) * 3,
                               log_probs=-np.abs(a[:n]).astype(np.float32),
                               stats=np.tile(np.array([1.0, 5.0, 0.5, 0.2], np.float32), (n, 1)),
                               T=3 * n + 1)

    def decode(self, chunks, beam=0):
        with self.lock:
            self.calls.append(len(chunks))
        return [self._one(c) for c in chunks]

    def decode_features(self, feats, beam=0):
        raise AssertionError("features path not expected")

    def fbank(self, a):
        return np.zeros((max(0, (len(a) + 80) // 160), 80), np.float32)


def _rec(h):
    toks = ["<blk>", "<sos/eos>", "<unk>"] + [f"▁w{i}" if i % 3 == 0 else f"p{i}" for i in range(3, 64)]
    return {"handle": h, "id2token": dict(enumerate(toks)), "vocab_size": 64, "max_active_paths": 8}


def _two_workers(rec, concat, plan):
    out = [None] * len(plan)

    def worker(idx):
        for i in idx:
            s, e, _ = plan[i]
            out[i] = ae.decode_chunk(rec, concat[s:e], s / 16000.0)

    ts = [threading.Thread(target=worker, args=(list(range(k, len(plan), 2)),)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def test_plan_registered_from_regions_equals_plan_chunks():
    audio = synth_speech(150.0, 7)
    assert ae.register_plan_from_regions(audio, silent_regions(audio), best_split)
    hit = ae._planned_span(audio[plan_chunks(audio)[2][0]:plan_chunks(audio)[2][1]])
    assert hit is not None
    assert hit[0].plan == [(s, e) for s, e, _ in plan_chunks(audio)]


def test_two_workers_served_by_one_batched_decode():
    concat = synth_speech(200.0, 11)
    plan = plan_chunks(concat)
    assert len(plan) >= 6
    direct = FakeHandle()
    want = [ae.decode_chunk(_rec(direct), concat[s:e].copy(), s / 16000.0) for s, e, _ in plan]
    assert direct.calls == [1] * len(plan)  # copies are not views of a planned signal
    h = FakeHandle()
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    got = _two_workers(_rec(h), concat, plan)
    assert h.calls == [len(plan)], h.calls  # ONE batched call for the whole plan
    assert got == want
    # a second pass (e.g. the reference's retry of failed chunks) reuses the results
    again = [ae.decode_chunk(_rec(h), concat[s:e], s / 16000.0) for s, e, _ in plan]
    assert h.calls == [len(plan)] and again == want


def test_unplanned_spans_and_disabled_routing_take_the_per_chunk_path(monkeypatch):
    concat = synth_speech(120.0, 12)
    plan = plan_chunks(concat)
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    h = FakeHandle()
    s, e, _ = plan[1]
    ae.decode_chunk(_rec(h), concat[s + 1:e], 0.0)  # not a span of the plan
    assert h.calls == [1]
    monkeypatch.setenv("ZASR_PLAN_AHEAD", "0")
    h2 = FakeHandle()
    ae.decode_chunk(_rec(h2), concat[s:e], 0.0)
    assert h2.calls == [1]


def test_precomputed_features_route_only_for_our_fbank_of_that_chunk(monkeypatch):
    concat = synth_speech(100.0, 13)
    plan = plan_chunks(concat)
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    h = FakeHandle()
    monkeypatch.setattr(ae, "_last_handle", h)
    s, e, _ = plan[0]
    feats = ae.compute_fbank_ort(concat[s:e])
    ae.decode_chunk(_rec(h), concat[s:e], 0.0, precomputed_features=feats)
    assert h.calls == [len(plan)]
    other = np.zeros_like(feats)  # features of unknown origin: the per-chunk features path
    h2 = FakeHandle()
    try:
        ae.decode_chunk(_rec(h2), concat[s:e], 0.0, precomputed_features=other)
        raise RuntimeError("expected the features path")
    except AssertionError as ex:
        assert "features path" in str(ex)


def test_dead_signal_is_not_matched():
    a = synth_speech(70.0, 14)
    ae.register_plan_from_regions(a, silent_regions(a), best_split)
    ptr = a.__array_interface__["data"][0]
    del a
    b = np.zeros(70 * 16000, np.float32)
    if b.__array_interface__["data"][0] == ptr:  # same address reused: still no match
        assert ae._planned_span(b[: 30 * 16000]) is None


def test_registration_starts_the_plan_decode_for_loaded_recognizers(monkeypatch):
    """The reference loads its recognizer(s) before it plans (:2041-2057): registering the plan
    starts their batched decode at once (a background thread), so the GPU works while the
    caller still builds its boundary list; the workers' calls then wait on that one decode."""
    concat = synth_speech(150.0, 15)
    plan = plan_chunks(concat)
    h = FakeHandle()
    rec = _rec(h)
    monkeypatch.setattr(ae, "_recognizer_cache", {("m", 8): rec})
    monkeypatch.setattr(ae, "_last_handle", h)
    assert ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    sig = ae._planned_span(concat[plan[0][0]:plan[0][1]])[0]
    sig.jobs[h][8].thread.join(timeout=30)
    assert h.calls == [len(plan)]  # decoded before any decode_chunk call
    got = _two_workers(rec, concat, plan)
    assert h.calls == [len(plan)]
    want = [ae.decode_chunk(rec, concat[s:e].copy(), s / 16000.0) for s, e, _ in plan]
    assert got == want


def test_silent_regions_from_flags_equals_the_reference_restatement():
    """regions_from_flags (the tail the GPU planner runs on zasr_silence_flags' output) gives
    the restated find_silent_regions' regions; pinned by plan_cases.json through
    test_host_plan_rover.  Edge cases: leading / trailing silence, runs of exactly 29 / 30
    frames (int(0.3 / 0.01) = 29), a signal shorter than one frame."""
    from zasr.plan import regions_from_flags
    rng = np.random.default_rng(3)
    for n_frames, pattern in [(400, "edges"), (1000, "random"), (0, "none")]:
        a = (rng.standard_normal(n_frames * 160 + 37) * 0.05).astype(np.float32)
        if pattern == "edges":
            a[:50 * 160] *= 0.01
            a[-45 * 160:] *= 0.01
            a[100 * 160:129 * 160] *= 0.01  # 29 quiet frames: a region
            a[200 * 160:228 * 160] *= 0.01  # 28: not
        elif pattern == "random":
            for s in rng.integers(0, n_frames - 40, 20):
                a[s * 160:(s + int(rng.integers(10, 40))) * 160] *= 0.01
        nf = len(a) // 160
        rms = np.sqrt(np.mean(a[:nf * 160].reshape(nf, 160) ** 2, axis=1))
        assert regions_from_flags(rms < 0.01, 160, len(a)) == silent_regions(a)


class FailingBatchHandle(FakeHandle):
    """Batched decodes fail (e.g. out of HBM for a long plan), single chunks succeed."""

    def decode(self, chunks, beam=0):
        if len(chunks) > 1:
            with self.lock:
                self.calls.append(-len(chunks))
            raise RuntimeError("hipErrorOutOfMemory (stand-in)")
        return super().decode(chunks, beam)


def test_failed_plan_decode_falls_back_to_the_per_chunk_path(caplog):
    """a failed plan decode must not fail every chunk of the plan: it is logged
    once and each chunk decodes on its own, with the per-chunk words."""
    concat = synth_speech(160.0, 16)
    plan = plan_chunks(concat)
    want = [ae.decode_chunk(_rec(FakeHandle()), concat[s:e].copy(), s / 16000.0)
            for s, e, _ in plan]
    h = FailingBatchHandle()
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    with caplog.at_level("WARNING", logger="zasr.asr_engine"):
        got = _two_workers(_rec(h), concat, plan)
    assert got == want
    assert h.calls[0] == -len(plan) and h.calls.count(1) == len(plan)
    assert sum("plan decode failed" in r.getMessage() for r in caplog.records) == 1


def test_eager_start_only_for_the_last_used_recognizer_or_the_rover_pair(monkeypatch):
    """a second cached recognizer of an earlier model is not decoded eagerly; the
    ROVER pair (both models used per chunk, :2346-2350) is."""
    concat = synth_speech(90.0, 17)
    plan = plan_chunks(concat)
    old, cur = FakeHandle(), FakeHandle()
    r_old, r_cur = _rec(old), _rec(cur)
    r_old["model_path"], r_cur["model_path"] = "/m/other-model", "/m/current-model"
    monkeypatch.setattr(ae, "_recognizer_cache", {("a", 8): r_old, ("b", 8): r_cur})
    monkeypatch.setattr(ae, "_last_handle", cur)
    assert [h for h, _ in ae._eager_handles()] == [cur]
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
    sig = ae._planned_span(concat[plan[0][0]:plan[0][1]])[0]
    sig.jobs[cur][8].thread.join(timeout=30)
    assert cur.calls == [len(plan)] and old.calls == [] and old not in sig.jobs
    # the earlier model still gets the plan's batch on its first planned chunk
    s, e, _ = plan[0]
    ae.decode_chunk(r_old, concat[s:e], 0.0)
    assert old.calls == [len(plan)]
    a, b = FakeHandle(), FakeHandle()
    ra, rb = _rec(a), _rec(b)
    ra["model_path"] = "/models/" + ae.ROVER_MODEL_IDS[0]
    rb["model_path"] = "/models/" + ae.ROVER_MODEL_IDS[1] + "/"
    monkeypatch.setattr(ae, "_recognizer_cache", {("a", 8): ra, ("b", 8): rb})
    assert {id(h) for h, _ in ae._eager_handles()} == {id(a), id(b)}


def test_wpe_caller_registers_without_decoding(monkeypatch):
    """With preprocess_wpe the workers decode WPE copies (:2338-2341): the hook registers the
    plan but starts no decode (zasr.dropin._caller_uses_wpe reads the caller's config)."""
    from zasr.dropin import _caller_uses_wpe
    concat = synth_speech(80.0, 18)
    h = FakeHandle()
    monkeypatch.setattr(ae, "_recognizer_cache", {("m", 8): _rec(h)})
    monkeypatch.setattr(ae, "_last_handle", h)

    class Pipe:
        def __init__(self, wpe):
            self.config = {"preprocess_wpe": wpe}

        def plan(self):
            import sys
            return _caller_uses_wpe(sys._getframe(0))

    assert Pipe(True).plan() and not Pipe(False).plan()
    assert ae.register_plan_from_regions(concat, silent_regions(concat), best_split, start=False)
    sig = ae._planned_span(concat[: plan_chunks(concat)[0][1]])[0]
    assert h not in sig.jobs and h.calls == []


def test_hbm_copy_released_after_the_decode_and_entry_pruned_with_the_signal(monkeypatch):
    """the plan's HBM copy of the signal is dropped once its decode has finished,
    and the registry entry goes when the pipeline drops the signal (weakref callback)."""
    import gc
    concat = synth_speech(75.0, 19)
    plan = plan_chunks(concat)
    h = FakeHandle()
    monkeypatch.setattr(ae, "_recognizer_cache", {("m", 8): _rec(h)})
    monkeypatch.setattr(ae, "_last_handle", h)
    marker = SimpleNamespace(device=SimpleNamespace(index=-1))  # an HBM copy on another device
    ae.register_plan_from_regions(concat, silent_regions(concat), best_split, d_audio=marker)
    sig = ae._planned_span(concat[plan[0][0]:plan[0][1]])[0]
    sig.jobs[h][8].thread.join(timeout=30)
    assert sig.d_audio is None and h.calls == [len(plan)]
    n_before = len(ae._planned)
    del concat
    gc.collect()
    assert sig not in ae._planned and len(ae._planned) == n_before - 1
