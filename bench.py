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


def gemm_flops(cfg, L_list):
    """Algorithmic FLOPs of the encoder's dense projections + frontend convs (as GEMMs)."""
    f_enc = 0.0
    for L in L_list:
        T = 2 * L + 7
        L2 = (T - 3) // 2
        f_enc += 2.0 * (L2 * 39 * 72 * 32 + L * 19 * 288 * 128 + 2 * L * 19 * 128 * 384
                        + L * 2432 * cfg.encoder_dims[0])
        for i, d in enumerate(cfg.encoder_dims):
            R = -(-L // cfg.downsampling[i])
            F, h = cfg.ff_dims[i], cfg.num_heads[i]
            hid = 3 * d // 4
            per_row = ((2 * cfg.query_head_dim + cfg.pos_head_dim) * h * d
                       + 2 * (2 * cfg.value_head_dim * h * d)
                       + 2 * ((F * 3) // 4 + F + (F * 5) // 4) * d
                       + 3 * hid * d + hid * d + 2 * (2 * d * d + d * d))
            f_enc += 2.0 * R * per_row * cfg.num_layers[i]
        f_enc += 2.0 * ((L + 1) // 2) * cfg.max_dim * cfg.joiner_dim
    return f_enc


def attn_bytes(cfg, L_list):
    """HBM bytes of the materialised attention weights: 1 write + 3 reads (nonlin head 0,
    self_attn1, self_attn2) per layer, f32."""
    w = r = 0.0
    for L in L_list:
        for i in range(cfg.num_stacks):
            R = -(-L // cfg.downsampling[i])
            R4 = (R + 3) // 4 * 4
            per = 4.0 * cfg.num_heads[i] * R * R4 * cfg.num_layers[i]
            w += per
            r += per * 2 + per / cfg.num_heads[i]
    return w, r


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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="zipformer-68m")
    ap.add_argument("--method", default="greedy_search")
    ap.add_argument("--beam", type=int, default=8)
    ap.add_argument("--audio-sec", type=float, default=3600.0)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    rec = Recognizer(mdir, args.method, beam, device_id=local, precision=args.precision)

    # per-rank shard: the same hour of synthetic audio, seeded by rank
    chunks = make_chunks(args.audio_sec, 20261015 + rank)
    lens = [c.shape[0] for c in chunks]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    d_wav = torch.from_numpy(np.concatenate(chunks)).to(f"cuda:{local}")
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        return rec.decode_device(d_wav.data_ptr(), offs, lens, beam=beam, stream=stream)

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()

    # timed region: barrier + sync on both sides, max over ranks
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
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
    f_gemm = gemm_flops(cfg, L_list)
    aw, ar = attn_bytes(cfg, L_list)
    rows_joiner = sum(min(beam, 8) * ((L + 1) // 2) for L in L_list)
    f_join = 2.0 * rows_joiner * cfg.joiner_dim * cfg.vocab_size
    classes = {k: v for k, v in prof.items()}
    dom = max(classes.items(), key=lambda kv: kv[1][1])[0] if classes else None
    peak_mfma = MFMA_F32_PEAK_TFLOPS if args.precision == "fp32" else MFMA_BF16_PEAK_TFLOPS
    roof = None
    if dom:
        cnt, ms = classes[dom]
        per_launch_ms = ms / cnt
        if dom in ("enc_gemm", "frontend_conv"):
            work = f_gemm * nprof / cnt  # FLOPs per launch (class average)
            ach = work / (per_launch_ms * 1e-3) / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2),
                    "peak": peak_mfma, "unit": "TFLOP/s", "frac": round(ach / peak_mfma, 4),
                    "traffic": None}
        elif dom == "joiner":
            work = f_join * nprof / cnt
            ach = work / (per_launch_ms * 1e-3) / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2),
                    "peak": peak_mfma, "unit": "TFLOP/s", "frac": round(ach / peak_mfma, 4),
                    "traffic": None}
        elif dom in ("attn_apply", "attn_softmax"):
            b = (ar if dom == "attn_apply" else aw) * nprof / cnt
            ach = b / (per_launch_ms * 1e-3) / 1e9
            roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": None}
        else:
            roof = {"kernel": dom, "bound": "latency", "achieved": None, "peak": None,
                    "unit": None, "frac": None, "traffic": None}
        roof["avg_launch_ms"] = round(per_launch_ms, 4)
        roof["launches_per_step"] = cnt // nprof

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
                                   f"{'' if beam == 1 else ' beam %d' % beam}, batched VAD-style chunks",
                       "model": args.model, "chunks_per_gpu": len(chunks),
                       "audio_sec_per_gpu": audio_sec_rank,
                       "decoded_sec_per_gpu_incl_overlap": round(decoded_sec_rank, 1),
                       "parallelism": f"dp{world} (chunk shards, no collective)",
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
