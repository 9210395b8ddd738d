"""The reference's unchanged two-worker loop through the drop-in decode_chunk on an MI355X
(core/asr_engine.py:2219-2237, 2326-2397): with the plan registered (the find_silent_regions
hook of zasr.dropin), every chunk's words come from ONE batched decode of the plan and equal
the per-chunk path's words exactly (tokens, timestamps, probabilities, entropy fields); the
ROVER route (compute_fbank_ort once per chunk, decode_chunk with precomputed_features,
:2346-2350) likewise."""
import threading

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dropin_rec():
    if not gpu_available():
        pytest.skip("no GPU")
    from model_fixtures import m_model
    from zasr import asr_engine as ae
    cfg, w, path = m_model()
    rec = ae.create_recognizer(path, 4, max_active_paths=8, hotwords=([], []), precision="bf16x3")
    yield ae, rec
    ae.clear_model_cache()


def _loop(ae, rec, concat, plan, feats=False):
    out = [None] * len(plan)
    errs = []

    def worker(idx):
        try:
            for i in idx:
                s, e, _ = plan[i]
                c = concat[s:e]
                f = ae.compute_fbank_ort(c, 16000) if feats else None
                out[i] = ae.decode_chunk(rec, c, s / 16000.0, precomputed_features=f)
        except Exception as ex:  # pragma: no cover - surfaced below
            errs.append(ex)

    ts = [threading.Thread(target=worker, args=(list(range(k, len(plan), 2)),)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return out


def _calls(h):
    """Count the handle's decode / decode_features calls."""
    n = {"decode": 0, "feat": 0, "chunks": 0}
    d0, f0 = h.decode, h.decode_features

    def dec(chunks, beam=0):
        n["decode"] += 1
        n["chunks"] += len(chunks)
        return d0(chunks, beam=beam)

    def decf(feats, beam=0):
        n["feat"] += 1
        return f0(feats, beam=beam)
    h.decode, h.decode_features = dec, decf
    return n


@pytest.mark.parametrize("feats", [False, True], ids=["audio", "rover_features"])
def test_two_worker_loop_routed_equals_per_chunk(dropin_rec, feats):
    from zasr.plan import best_split, plan_chunks, silent_regions
    from zasr.synth_audio import synth_speech
    ae, rec = dropin_rec
    concat = synth_speech(170.0, 31 + int(feats))
    plan = plan_chunks(concat)
    assert len(plan) >= 5
    h = rec["handle"]
    n = _calls(h)
    try:
        want = [ae.decode_chunk(rec, concat[s:e].copy(), s / 16000.0) for s, e, _ in plan]
        assert n["decode"] == len(plan)
        n["decode"] = n["feat"] = 0  # before registering: the plan's decode starts there
        assert ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
        got = _loop(ae, rec, concat, plan, feats)
        assert n["decode"] == 1 and n["feat"] == 0, n  # one batched pass for the whole plan
    finally:
        del h.decode, h.decode_features
    assert sum(len(w) for w in want) > 50
    assert got == want


def test_failed_plan_decode_falls_back_per_chunk(dropin_rec):
    """the plan's batched decode raising (e.g. out of HBM) must not break
    the caller -- every decode_chunk of the two-worker loop then takes the per-chunk path and
    returns the per-chunk words."""
    from zasr.plan import best_split, plan_chunks, silent_regions
    from zasr.synth_audio import synth_speech
    ae, rec = dropin_rec
    concat = synth_speech(120.0, 57)
    plan = plan_chunks(concat)
    assert len(plan) >= 3
    h = rec["handle"]
    want = [ae.decode_chunk(rec, concat[s:e].copy(), s / 16000.0) for s, e, _ in plan]
    d0 = h.decode
    calls = {"batched": 0, "single": 0}

    def failing(chunks, beam=0):
        if len(chunks) > 1:  # the plan's batched pass
            calls["batched"] += 1
            raise RuntimeError("injected: HIP out of memory in the plan decode")
        calls["single"] += 1
        return d0(chunks, beam=beam)
    h.decode = failing
    try:
        assert ae.register_plan_from_regions(concat, silent_regions(concat), best_split)
        got = _loop(ae, rec, concat, plan)
    finally:
        del h.decode
    assert calls["batched"] == 1 and calls["single"] == len(plan), calls
    assert got == want


def test_decode_sharded_real_recognizer_nccl_world1(dropin_rec):
    """zasr.shard.decode_sharded with a real Recognizer under an initialised RCCL ("nccl")
    process group of size 1: the LPT split, the decode and the all_gather_object of the word
    lists (pickled through device tensors) run once on the GPU; the words equal decode_chunk's
    per chunk."""
    import socket

    import torch.distributed as dist
    from zasr.plan import plan_chunks
    from zasr.synth_audio import synth_speech
    ae, rec = dropin_rec
    audio = synth_speech(95.0, 77)
    plan = plan_chunks(audio)
    chunks = [audio[s:e].copy() for s, e, _ in plan]
    offs = [s / 16000.0 for s, _, _ in plan]
    want = [ae.decode_chunk(rec, c, o) for c, o in zip(chunks, offs)]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    import torch
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        got = ae.decode_chunks(rec, chunks, offs)
    finally:
        dist.destroy_process_group()
    assert got == want
    assert sum(len(w) for w in got) > 20


def _np_flags(a, flen, thr=0.01):
    nf = len(a) // flen
    return np.sqrt(np.mean(a[:nf * flen].reshape(nf, flen) ** 2, axis=1)) < thr


@pytest.mark.parametrize("flen", [160, 80, 240, 128, 136])
def test_silence_flags_bit_exact_vs_numpy(flen):
    """zasr_silence_flags against numpy's own float32 evaluation of find_silent_regions'
    energies < threshold (core/asr_engine.py:526-536), with frames placed within a few ulps
    of the threshold (RMS = 0.01 * (1 + k * 2^-24)) where any other summation order, an FMA
    contraction or a float64 comparison flips the flag."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from zasr.binding import silence_flags
    rng = np.random.default_rng(flen)
    nf = 20000
    a = (rng.standard_normal(nf * flen + 50) * 0.02).astype(np.float32)
    for f in range(0, nf, 3):  # two thirds of the frames right at the threshold
        row = rng.standard_normal(flen).astype(np.float64)
        row *= 0.01 * (1.0 + rng.integers(-40, 41) * 2.0 ** -24) / np.sqrt(np.mean(row ** 2))
        a[f * flen:(f + 1) * flen] = row.astype(np.float32)
    d = torch.from_numpy(a).cuda()
    flags = torch.zeros(nf, dtype=torch.uint8, device="cuda")
    silence_flags(d.data_ptr(), len(a), flen, 0.01, flags.data_ptr())
    got = flags.cpu().numpy().astype(bool)
    want = _np_flags(a, flen)
    assert 0.1 < want.mean() < 0.5  # a sixth of the frames below the threshold
    assert np.array_equal(got, want), int((got != want).sum())


def test_gpu_planner_routes_the_two_worker_loop(dropin_rec):
    """The drop-in's find_silent_regions route: the regions from the GPU silence detector
    equal the reference's (restated, plan_cases-pinned) find_silent_regions; the plan's
    decode starts at registration from the HBM copy of the signal (one
    decode_device_batches call, no host upload, no per-chunk decode) and the two workers'
    decode_chunk words equal the per-chunk path's."""
    from zasr.plan import best_split, plan_chunks, silent_regions
    from zasr.synth_audio import synth_speech
    ae, rec = dropin_rec
    concat = synth_speech(260.0, 41)
    plan = plan_chunks(concat)
    h = rec["handle"]
    want = [ae.decode_chunk(rec, concat[s:e].copy(), s / 16000.0) for s, e, _ in plan]
    n = _calls(h)
    nb = {"batches": 0}
    b0 = h.decode_device_batches

    def dev_batches(*a, **k):
        nb["batches"] += 1
        return b0(*a, **k)
    h.decode_device_batches = dev_batches
    try:
        regions = ae.plan_ahead_regions(concat, best_split)
        assert regions == silent_regions(concat)
        got = _loop(ae, rec, concat, plan)
        assert nb["batches"] == 1 and n["decode"] == 0 and n["feat"] == 0, (nb, n)
    finally:
        del h.decode, h.decode_features, h.decode_device_batches
    assert sum(len(w) for w in want) > 50
    assert got == want
