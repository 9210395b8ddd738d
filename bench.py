"""Benchmark: Zipformer-68M offline decode throughput (audio-seconds per second, xRT).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model zipformer-68m]
                    [--method greedy_search|modified_beam_search] [--beam 8]
                    [--audio-sec 3600] [--no-cpu-baseline]

One step = one pass of the hot path (fbank -> Conv2dSubsampling -> Zipformer2 encoder ->
decoder/joiner -> search) over one batch of synthetic 16 kHz speech: `--audio-sec` seconds
(default 1 h) cut by the reference planner into ~30 s chunks with 3 s overlap
(core/asr_engine.py:2137-2161), all chunks decoded in one batched pass per GPU.  The
waveforms are resident in HBM before the timed region.  N > 1: one process per GPU
(torch.distributed.run), each rank decodes its own 1 h shard (weak scaling, no data-path
collective); the time is the max over ranks.

Prints one JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "sherpa-vietnamese-asr_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

SR = 16000
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md chip table (f32-input MFMA)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense
HBM_PEAK_GBS = 8000.0


def make_chunks(audio_sec: float, seed: int):
    """~30 s chunks (+3 s overlap) of seeded synthetic speech: windows of a 5-minute base
    signal with per-chunk gain and noise (cheap to build for an hour of audio)."""
    from zasr.synth_audio import chunk_plan, synth_speech
    total = int(audio_sec * SR)
    base = synth_speech(min(audio_sec, 300.0) + 40.0, seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    chunks = []
    for a, e, _ in chunk_plan(total):
        n = e - a
        s = int(rng.integers(0, base.shape[0] - n))
        c = base[s:s + n] * np.float32(rng.uniform(0.7, 1.1))
        c = c + np.float32(1e-3) * rng.standard_normal(n).astype(np.float32)
        chunks.append(np.ascontiguousarray(c, dtype=np.float32))
    return chunks


FFN_FUSED_DIMS = (64, 96, 128, 192)  # ffn_kernels.hip ffn_fused_supported


def gemm_class_work(cfg, L_list, bf16: bool):
    """Algorithmic work per step of the GEMM-class launches, mirroring Engine::run_encoder /
    layer_forward: {"enc_gemm": (flops, bytes), "ffn_fused": (flops, bytes)}.

    enc_gemm = every Engine::linear / linear_h (stack projections, embed out, encoder_proj;
    in the fp32 mode also the ConvNeXt pointwise convs).  Bytes per launch = A read + weights
    + C write (+ C read for the residual epilogue), each at the dtype the launch really uses
    (bf16 mode: GEMM -> GEMM intermediates, q/k/v and the hidden activations in bf16; the
    residual stream f32).  ffn_fused (bf16 mode, model dim in FFN_FUSED_DIMS) = X read + X
    written (f32) + both weight matrices (bf16), 4 R d F flops."""
    wb = 2 if bf16 else 4
    acc = {"enc_gemm": [0.0, 0.0], "ffn_fused": [0.0, 0.0]}

    def lin(M, K, N, a=4, c=4, resadd=False):
        if M <= 0:
            return
        acc["enc_gemm"][0] += 2.0 * M * K * N
        acc["enc_gemm"][1] += a * M * K + wb * N * K + c * M * N * (2 if resadd else 1)

    h16 = 2 if bf16 else 4  # intermediates stored in bf16 in the bf16 mode
    d0 = cfg.encoder_dims[0]
    Ls = [L for L in L_list if L > 0]
    Lsum = sum(Ls)
    if bf16:
        lin(Lsum, 128 * 19, d0, a=2)  # embed out over the bf16 ConvNeXt output
    else:
        lin(19 * Lsum, 128, 384)
        lin(19 * Lsum, 384, 128, resadd=True)
        lin(Lsum, 128 * 19, d0)
    for i, d in enumerate(cfg.encoder_dims):
        R = sum(-(-L // cfg.downsampling[i]) for L in Ls)
        F, h = cfg.ff_dims[i], cfg.num_heads[i]
        hid = 3 * d // 4
        for _ in range(cfg.num_layers[i]):
            lin(R, d, (2 * cfg.query_head_dim + cfg.pos_head_dim) * h, c=h16)
            for f in ((F * 3) // 4, F, (F * 5) // 4):
                if bf16 and d in FFN_FUSED_DIMS:
                    acc["ffn_fused"][0] += 4.0 * R * d * f
                    acc["ffn_fused"][1] += 8.0 * R * d + 2 * 2.0 * f * d
                else:
                    lin(R, d, f, c=h16)
                    lin(R, f, d, a=h16, resadd=True)
            lin(R, d, 3 * hid)
            lin(R, hid, d, a=h16, resadd=True)
            for _ in range(2):
                lin(R, d, cfg.value_head_dim * h, c=h16)
                lin(R, cfg.value_head_dim * h, d, a=h16, resadd=True)
                lin(R, d, 2 * d, c=h16)
                lin(R, d, d, a=h16, resadd=True)
    lin(sum((L + 1) // 2 for L in Ls), cfg.max_dim, cfg.joiner_dim)
    return {k: (v[0], v[1]) for k, v in acc.items()}


def pmc_traffic(kernel_class, args):
    """HBM bytes per launch of the dominant class from a committed rocprofv3 PMC pass of this
    same configuration (tools/pmc_traffic.py writes it: FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE, MI355X_MICROARCH.md HBM section), or None."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    key = f"{args.model}|{args.method}|{args.beam if args.method != 'greedy_search' else 1}|" \
          f"{args.precision}|{int(args.audio_sec)}|{kernel_class}"
    return tab.get(key)


def cpu_baseline(model_dir_cfg, weights, chunks, method_beam, budget_s=20.0):
    """Oracle (fp32 torch encoder + numpy fbank + Python search) on a bounded sample."""
    import torch
    from oracle.fbank import fbank
    from oracle.search import beam_search
    from oracle.zipformer import ZipformerOracle
    try:
        import psutil
        phys = psutil.cpu_count(logical=False) or os.cpu_count()
    except Exception:
        phys = os.cpu_count()
    threads = max(1, min(phys, 16))  # reference policy: encoder Z = physical cores
    torch.set_num_threads(threads)
    orc = ZipformerOracle(model_dir_cfg, weights)
    done_sec, t0, used = 0.0, time.time(), 0
    # warm-up (reference calibration: 1 warmup then measured runs, core/calibration.py:822-830)
    orc.encoder(fbank(chunks[0][: SR * 3]))
    t0 = time.time()
    for c in chunks:
        enc = orc.encoder(fbank(c))
        beam_search(enc, orc.decoder, orc.joiner, method_beam)
        done_sec += c.shape[0] / SR
        used += 1
        if time.time() - t0 > budget_s:
            break
    el = time.time() - t0
    return {"value": round(done_sec / el, 3), "unit": "audio-sec/sec", "cores": threads,
            "kind": "port",
            "sample": f"{used} chunk(s), {done_sec:.1f} s of the same synthetic audio, "
                      f"oracle fbank+encoder+{'greedy' if method_beam == 1 else 'beam %d' % method_beam}"
                      f" search, torch fp32 {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="zipformer-68m")
    ap.add_argument("--method", default="greedy_search")
    ap.add_argument("--beam", type=int, default=8)
    ap.add_argument("--audio-sec", type=float, default=3600.0)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "bf16_enc", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hotwords", type=int, default=0,
                    help="N synthetic hotwords (2-4 tokens each, score 1.5 as the reference's "
                         "hotwords_score default, core/asr_engine.py:1000); beam search only")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="steps as separate decode_device calls (no cross-batch overlap)")
    ap.add_argument("--profile-out", default="")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)

    from zasr.binding import Recognizer
    from zasr.model import PRESETS, save_model_dir, synth_tokens, synth_weights

    cfg = PRESETS[args.model]()
    weights = synth_weights(cfg, 20261015)
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_bench_{args.model}_{os.getpid()}")
    save_model_dir(mdir, cfg, weights, synth_tokens(cfg.vocab_size))
    beam = 1 if args.method == "greedy_search" else args.beam
    hotwords = None
    if args.hotwords:
        hr = np.random.default_rng(20261016)
        hotwords = [hr.integers(1, cfg.vocab_size, size=int(hr.integers(2, 5))).tolist()
                    for _ in range(args.hotwords)]
    rec = Recognizer(mdir, args.method, beam, hotwords=hotwords, device_id=local,
                     precision=args.precision)

    # per-rank shard: the same hour of synthetic audio, seeded by rank
    chunks = make_chunks(args.audio_sec, 20261015 + rank)
    lens = [c.shape[0] for c in chunks]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    d_wav = torch.from_numpy(np.concatenate(chunks)).to(f"cuda:{local}")
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        return rec.decode_device(d_wav.data_ptr(), offs, lens, beam=beam, stream=stream)

    def steps(k):
        # k steps = k consecutive batches (each the hour of chunks) through the engine's
        # batch pipeline: batch i+1's fbank + encoder overlap batch i's search on the GPU
        # (zasr_decode_device_batches); every batch's results are complete on return
        if args.no_pipeline:
            for _ in range(k):
                r = step()
            return r
        n = len(lens)
        r = rec.decode_device_batches(d_wav.data_ptr(), offs * k, lens * k, [n] * k,
                                      beam=beam, stream=stream)
        return r[-n:]

    if args.warmup:
        res = steps(args.warmup)
    torch.cuda.synchronize()
    # single-batch latency (one hour of chunks, nothing to overlap with): reported beside
    t1 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    batch_latency_ms = 1000 * (time.perf_counter() - t1)

    # timed region: barrier + sync on both sides, max over ranks
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = steps(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
        dist.barrier()

    # kernel-class timing: HIP events recorded by the library on its launch stream over
    # K profiled steps (separate from the wall-clock region above)
    rec.profile(True)
    rec.profile_reset()
    for _ in range(max(1, min(args.steps, 3))):
        step()
    torch.cuda.synchronize()
    prof = rec.profile_report()
    rec.profile(False)
    nprof = max(1, min(args.steps, 3))

    audio_sec_rank = args.audio_sec
    decoded_sec_rank = sum(lens) / SR
    value = audio_sec_rank * world * args.steps / el
    emitted = sum(int(r.token_ids.size) for r in res)
    tprime = sum(int(r.T) for r in res)

    L_list = [((n + 80) // 160 - 7) // 2 for n in lens]
    bf16 = args.precision == "bf16"
    work = gemm_class_work(cfg, L_list, bf16)
    rows_joiner = sum(min(beam, 8) * ((L + 1) // 2) for L in L_list)
    f_join = 2.0 * rows_joiner * cfg.joiner_dim * cfg.vocab_size
    classes = {k: v for k, v in prof.items()}
    dom = max(classes.items(), key=lambda kv: kv[1][1])[0] if classes else None
    peak_mfma = MFMA_BF16_PEAK_TFLOPS if bf16 else MFMA_F32_PEAK_TFLOPS
    roof = None
    if dom:
        cnt, ms = classes[dom]
        per_launch_s = ms / cnt * 1e-3
        if dom in work:
            # the binding roof is the larger of bytes / HBM peak and flops / MFMA peak
            f_cls, b_cls = work[dom]
            fl, by = f_cls * nprof / cnt, b_cls * nprof / cnt  # per launch (class mean)
            if by / (HBM_PEAK_GBS * 1e9) >= fl / (peak_mfma * 1e12):
                ach = by / per_launch_s / 1e9
                roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                        "algorithmic_bytes_per_launch": round(by),
                        "mfma_tflops": round(fl / per_launch_s / 1e12, 2)}
            else:
                ach = fl / per_launch_s / 1e12
                roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2),
                        "peak": peak_mfma, "unit": "TFLOP/s",
                        "frac": round(ach / peak_mfma, 4), "traffic": None,
                        "algorithmic_flops_per_launch": round(fl),
                        "hbm_gbs": round(by / per_launch_s / 1e9, 1)}
        elif dom == "joiner":
            work = f_join * nprof / cnt
            ach = work / per_launch_s / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2),
                    "peak": peak_mfma, "unit": "TFLOP/s", "frac": round(ach / peak_mfma, 4),
                    "traffic": None}
        else:
            # search step / decoder: one block per stream per frame, latency-bound
            roof = {"kernel": dom, "bound": "latency", "achieved": None, "peak": None,
                    "unit": None, "frac": None, "traffic": None}
        roof["avg_launch_ms"] = round(per_launch_s * 1e3, 4)
        roof["launches_per_step"] = cnt // nprof
        tr = pmc_traffic(dom, args)
        if tr is not None:
            roof["traffic"] = tr["bytes_per_launch"]
            roof["traffic_source"] = tr["source"]

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, weights, chunks[:6], beam)

    if rank == 0:
        line = {
            "metric": "audio-sec/sec (xRT) Zipformer-68M offline decode",
            "value": round(value, 2), "unit": "audio-sec/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (seeded 16 kHz speech-like audio, random-init Zipformer weights)",
            "config": {"workload": f"{args.model} {args.method}"
                                   f"{'' if beam == 1 else ' beam %d' % beam}"
                                   f"{' + %d hotwords' % args.hotwords if args.hotwords else ''}"
                                   ", batched VAD-style chunks",
                       "model": args.model, "chunks_per_gpu": len(chunks),
                       "audio_sec_per_gpu": audio_sec_rank,
                       "decoded_sec_per_gpu_incl_overlap": round(decoded_sec_rank, 1),
                       "parallelism": f"dp{world} (chunk shards, no collective)",
                       "batch_pipeline": not args.no_pipeline,
                       "single_batch_latency_ms": round(batch_latency_ms, 3),
                       "rtf": round(1.0 / (value / world), 6),
                       "tokens_emitted_per_gpu": emitted, "encoder_frames_per_gpu": tprime},
            "roofline": roof,
            "kernel_classes_ms_per_step": {k: round(v[1] / nprof, 3) for k, v in classes.items()},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    rec.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
