"""Benchmark: Zipformer-68M offline decode throughput (audio-seconds per second, xRT).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model zipformer-68m]
                    [--method greedy_search|modified_beam_search] [--beam 8]
                    [--hotwords-file default|PATH] [--audio-sec 3600]
                    [--precision bf16|bf16_enc|fp32] [--no-cpu-baseline] [--shape-table]

One step = one pass of the hot path (fbank -> Conv2dSubsampling -> Zipformer2 encoder ->
decoder/joiner -> search) over one batch: `--audio-sec` seconds (default 1 h) of seeded
synthetic 16 kHz speech cut by the reference planner (zasr/plan.py: silence-aligned ~30 s
chunks with a 3 s overlap, core/asr_engine.py:2137-2161), all chunks decoded in one batched
pass.  The waveforms are resident in HBM before the timed region; K steps are K consecutive
batches through the engine's batch pipeline (zasr_decode_device_batches).

--gpus N > 1 without RANK in the environment: this process starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child (before touching
the GPU) and exits with its return code.  Under torch.distributed each rank decodes its own
hour (seed + rank; weak scaling, no collective on the data path); the timed region is
bracketed by barriers and the time is the max over ranks.

Prints one JSON line (rank 0).  DESIGN.md §7 has the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

# hardware queues per process (HIP's default is 4): the batch pipeline keeps up to five
# streams busy (caller, two encoder streams, two beam searches), and streams beyond the queue
# count share queues in creation order -- 8 measured +3.6 % on the beam 8 line, neutral on
# greedy (profiles/r02/hw_queues).  Set before anything initialises HIP; <= 32 as the pool allows.
if os.environ.get("ZASR_HW_QUEUES"):  # explicit choice (A/B runs)
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["ZASR_HW_QUEUES"]
elif int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

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
WEIGHT_SEED = 20261015
AUDIO_SEED = 20261015
DEFAULT_HOTWORDS = os.path.join(REPO, "tests", "golden", "hotword_sample.txt")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="zipformer-68m")
    ap.add_argument("--method", default="greedy_search")
    ap.add_argument("--beam", type=int, default=8)
    ap.add_argument("--audio-sec", type=float, default=3600.0)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "bf16_enc", "fp32", "bf16x3", "bf16x6", "f16x3"])
    ap.add_argument("--parity-precision", default="f16x3",
                    choices=["none", "fp32", "bf16x6", "bf16x3", "f16x3"],
                    help="asr stage: also time this token-exact precision mode on the same "
                         "workload in the same run and report it as the line's `parity_mode` "
                         "(f16x3: fp16 hi + scaled lo pieces, three MFMAs per product, f32 "
                         "quality; bf16x6: six bf16 piece products), with the count of the "
                         "benched chunks whose tokens equal an exact-f32 (fp32 mode) decode of "
                         "the same hour")
    ap.add_argument("--parity-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the fp32 decode of the hour that parity_mode's "
                         "chunks_identical_to_fp32 is measured against")
    ap.add_argument("--parity-steps", type=int, default=0,
                    help="timed steps of the parity-mode line (default: --steps)")
    ap.add_argument("--weights", default="greedy-calibrated",
                    choices=["greedy-calibrated", "beam-calibrated"],
                    help="synthetic weight variant (zasr.model.WEIGHT_VARIANTS): greedy-calibrated "
                         "(default; ~18 %% of frames emit under greedy, ~6 %% under beam 8) or "
                         "beam-calibrated (peaked non-blank joiner rows: beam 8 emits at the greedy "
                         "rate, ~18 %%, as a trained model does; 68M only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub-lines", action="store_true",
                    help="skip the config-3 / config-4 f16x3 lines run in child processes beside "
                         "the default (config 2) line")
    ap.add_argument("--cpu-repeats", type=int, default=5,
                    help="CPU baseline: 1 warm-up then the mean of this many repeats "
                         "(core/calibration.py:822-830)")
    ap.add_argument("--hotwords-file", default="",
                    help="hotword phrases (reference hotword.txt format, score 1.5 default, "
                         "core/config.py:405-408); tokenized by the syllable hash (bpe.model is "
                         "absent).  'default' = tests/golden/hotword_sample.txt (the "
                         "reference's hotword.txt).  Beam search only.")
    ap.add_argument("--shard-plan", action="store_true",
                    help="strong scaling (BASELINE config 4's 'segments sharded across 8 GPUs'): "
                         "every rank plans the SAME hour, decodes its longest-processing-time "
                         "share of the chunks (zasr.shard.lpt_partition) and the results are "
                         "gathered to every rank in chunk order (host object gather) inside the "
                         "timed region; value = that hour x steps / max-over-ranks time")
    ap.add_argument("--proxy-ranks", type=int, default=0,
                    help="single-GPU proxy of --shard-plan at N ranks (implies --shard-plan, "
                         "world 1 only): decode the largest of the N LPT shares; value = the "
                         "hour x steps / that share's time, the strong-scaling ceiling of N "
                         "ranks before the gather (DESIGN.md §9)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="steps as separate decode_device calls (no cross-batch overlap)")
    ap.add_argument("--shape-table", action="store_true",
                    help="also time every encoder GEMM shape (HIP events) and emit the "
                         "per-shape roofline table")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="no GPU: exercise the launcher / rank / timing / JSON path with gloo "
                         "and a CPU stand-in step (tests/test_bench_launcher.py)")
    ap.add_argument("--profile-out", default="")
    ap.add_argument("--stage", default="asr",
                    choices=["asr", "campp", "vad", "pipe", "rover", "dropin"],
                    help="asr: the Zipformer decode (default, BASELINE metric); campp: the CAM++ "
                         "speaker-embedding stage of config 5 (1.5 s windows, 0.6 s step); vad: "
                         "Silero VAD probabilities + segments of the hour (core/asr_engine.py:2090); "
                         "pipe: BASELINE config 5, decode + merge + CAM++ embeddings + ViBERT "
                         "punctuation of the hour (zasr/pipeline.py); rover: BASELINE config 4, "
                         "30M + 68M decode of the hour + block vote + merge (zasr/rover.py); "
                         "dropin: the reference's two-worker decode_chunk loop over the hour "
                         "through the drop-in surface (plan-ahead batching, zasr/asr_engine.py)")
    ap.add_argument("--vad-files", type=int, default=1,
                    help="VAD stage: the hour split into this many files decoded in one call "
                         "(1 = the reference's single-file case; the recurrence is one "
                         "workgroup per file)")
    ap.add_argument("--rover-sub-batches", type=int, default=1,
                    help="ROVER stage: each model decodes the hour as this many pipelined batches "
                         "(measured 1 / 2 / 4 / 8: 143 / 136 / 171 / 245 ms per hour: every batch "
                         "adds a frame chain as long as its longest chunk)")
    ap.add_argument("--rover-passes-per-call", type=int, default=4,
                    help="ROVER and pipe stages: hours per decode call (consecutive batches of one call "
                         "share the batch pipeline, beam search with two searches in flight; the "
                         "vote of a call's hours overlaps the next call's decode).  Measured "
                         "(sub-batches, hours per call) = (2, 1) / (1, 2) / (1, 4) / (2, 2): "
                         "25.7k / 27.0k / 29.1k / 23.5k xRT (profiles/r02/rover)")
    ap.add_argument("--campp-batch", type=int, default=4096,
                    help="CAM++ windows per launch group (the reference batches 32 on CPU; "
                         "measured 512 -> 6000: 167 -> 123 ms per hour, profiles/r02/campp_batch)")
    args = ap.parse_args(argv)
    if args.proxy_ranks > 1:
        args.shard_plan = True
    return args


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """--gpus N > 1 outside torch.distributed: run N ranks under torch.distributed.run as a
    CHILD process (this process never initialised the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------ workload
def shard_share(lens, world, rank, proxy_ranks=0):
    """This rank's chunk indices under --shard-plan (zasr.shard.lpt_partition); with
    --proxy-ranks N on one GPU, the largest (critical) of the N shares."""
    from zasr.shard import lpt_partition
    if proxy_ranks > 1 and world == 1:
        parts = lpt_partition(lens, proxy_ranks)
        return max(parts, key=lambda ix: sum(lens[i] for i in ix))
    return lpt_partition(lens, world)[rank]


def make_chunks(audio_sec: float, seed: int):
    """`audio_sec` of seeded synthetic speech cut by the reference planner (silence-aligned
    ~30 s boundaries, 3 s overlap; zasr/plan.py restates core/asr_engine.py:2137-2161).  The
    synthetic pauses (0.3-2 s) are shorter than the 5 s VAD merge gap (:2117), so the whole
    signal is one VAD group and the concatenated speech is the signal itself."""
    from zasr.plan import plan_chunks
    from zasr.synth_audio import synth_speech
    audio = synth_speech(audio_sec, seed)
    return [np.ascontiguousarray(audio[a:e]) for a, e, _ in plan_chunks(audio)]


def load_hotwords(path: str, V: int):
    from zasr.hotword_context import parse_hotwords_file
    from zasr.model import hash_tokenize_phrases
    return hash_tokenize_phrases(parse_hotwords_file(path, 1.5), V)


HOUR_GOLDEN = os.path.join(REPO, "tests", "golden", "bench_hour_oracle.json")


def edit_distance(a, b) -> int:
    """Levenshtein distance between two token lists (token error rate numerator)."""
    if len(a) < len(b):
        a, b = b, a
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i]
        for j, y in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y)))
        prev = cur
    return prev[-1]


def hour_golden(args, beam, hotwords, chunks):
    """The oracle's token ids for the benched hour (tests/golden/bench_hour_oracle.json, made
    in the build container by tests/golden/make_bench_hour_golden.py: numpy fbank -> torch fp32
    encoder -> the reference's _ort_beam_search restated, core/asr_engine.py:1023-1153), or
    None when this run's workload is not the one the file holds.  Data only: nothing of the
    oracle runs here."""
    variant = getattr(args, "weights", "greedy-calibrated")
    path = HOUR_GOLDEN if variant == "greedy-calibrated" else \
        HOUR_GOLDEN.replace(".json", f"_{variant}.json")
    if args.model != "zipformer-68m" or args.audio_sec != 3600.0 or not os.path.exists(path):
        return None
    if beam == 1:
        key = "greedy"
    elif beam == 8 and hotwords and args.hotwords_file == "default":
        key = "beam8_hw"
    else:
        return None
    with open(path) as f:
        g = json.load(f)
    if [int(c.shape[0]) for c in chunks] != g["chunk_samples"]:
        return None
    import hashlib
    h = hashlib.sha256()
    for c in chunks:
        h.update(np.ascontiguousarray(c, dtype=np.float32).tobytes())
    if h.hexdigest()[:32] != g["audio_sha256_32"]:
        return None
    return key, g[key], path.replace("bench_hour_oracle", "bench_hour_audit")


HOUR_AUDIT = os.path.join(REPO, "tests", "golden", "bench_hour_audit.json")
ROVER_GOLDEN = os.path.join(REPO, "tests", "golden", "bench_hour_oracle_rover.json")


def rover_golden_checks(args, beam, phrases, chunks, toks):
    """Config 4: each ROVER model's tokens of every timed pass vs the oracle's decode of the
    hour (data only: the golden file), or None when this run is not the golden's workload."""
    if (args.audio_sec != 3600.0 or beam != 8 or args.hotwords_file != "default" or
            not os.path.exists(ROVER_GOLDEN)):
        return None
    with open(ROVER_GOLDEN) as f:
        g = json.load(f)
    if [int(c.shape[0]) for c in chunks] != g["chunk_samples"]:
        return None
    import hashlib
    h = hashlib.sha256()
    for c in chunks:
        h.update(np.ascontiguousarray(c, dtype=np.float32).tobytes())
    if h.hexdigest()[:32] != g["audio_sha256_32"]:
        return None
    audit = ROVER_GOLDEN.replace("bench_hour_oracle", "bench_hour_audit")
    return {m: oracle_agreement(f"{m}_beam8_hw", g[f"{m}_beam8_hw"], [t[i] for t in toks], audit)
            for i, m in enumerate(("rover30m", "rover68m"))}



def oracle_agreement(key, ref, got_steps, audit_path=HOUR_AUDIT):
    """Token agreement of every timed step's decode (a list of per-chunk token lists per step)
    with the oracle golden: chunks identical (worst step), token error rate of the last step,
    and whether every differing chunk is one of the audited f32 ties of
    tests/golden/bench_hour_audit.json (tests/golden/make_bench_hour_audit.py: an oracle
    margin at the f32 rounding of the hypothesis scores, or an exact beam-boundary tie)
    decoding to the audited tokens."""
    same = [sum(a == b for a, b in zip(got, ref)) for got in got_steps]
    last = got_steps[-1]
    errs = sum(edit_distance(a, b) for a, b in zip(last, ref))
    nref = sum(len(t) for t in ref)
    diff = [i for i, (a, b) in enumerate(zip(last, ref)) if a != b]
    audited = None
    if os.path.exists(audit_path):
        with open(audit_path) as f:
            au = json.load(f).get(key, {})
        ok = set(au.get("allowed_chunks", []))
        audited = all(i in ok and got[i] in au["chunks"][str(i)]["gpu_tokens"].values()
                      for got in got_steps for i, (a, b) in enumerate(zip(got, ref)) if a != b)
    gname = os.path.basename(audit_path).replace("bench_hour_audit", "bench_hour_oracle")
    return {"golden": f"tests/golden/{gname}[{key}]",
            "chunks_identical_to_oracle": f"{min(same)}/{len(ref)}",
            "per_timed_step": same if len(same) <= 32 else same[:32],
            "oracle_tokens": nref, "token_errors": errs,
            "ter": round(errs / max(1, nref), 5),
            "differing_chunks": diff[:24],
            "differing_chunks_all_audited_f32_ties": audited}


FFN_FUSED_DIMS = (64, 96, 128, 192, 256, 384, 512)  # ffn_kernels.hip ffn_fused_supported


def ffn_fused(d: int, f: int) -> bool:
    """Engine::layer_forward's choice: the fused FFN (ffn_fused_kernel up to 192,
    ffn_wide_kernel from 256 with F a multiple of 32 up to 2048)."""
    return d in FFN_FUSED_DIMS and (d < 256 or (f % 32 == 0 and f <= 2048))


def ffn_fused_h3(d: int, f: int) -> bool:
    """The f16x3 mode's fused FFN (ffn_kernels.hip ffn_h3_supported)."""
    return (d in (256, 384, 512) and f % 32 == 0 and f >= 32) or (d == 192 and f % 64 == 0)


def gemm_class_work(cfg, L_list, bf16: bool, h3: bool = False):
    """Algorithmic work per step of the GEMM-class launches, mirroring Engine::run_encoder /
    layer_forward: {"enc_gemm": (flops, bytes), "ffn_fused": (flops, bytes)}.

    enc_gemm = every Engine::linear / linear_h (stack projections, embed out, encoder_proj;
    in the fp32 mode also the ConvNeXt pointwise convs).  Bytes per launch = A read + weights
    + C write (+ C read for the residual epilogue), each at the dtype the launch really uses
    (bf16 mode: GEMM -> GEMM intermediates, q/k/v and the hidden activations in bf16; the
    residual stream f32).  ffn_fused (bf16 mode, model dim in FFN_FUSED_DIMS) = X read + X
    written (f32) + both weight matrices (bf16), 4 R d F flops.  h3: the f16x3 mode, whose
    FFNs (ffn_fused_h3 dims) are the fused f16x3 kernel (weights as two fp16 pieces)."""
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
                if bf16 and ffn_fused(d, f):
                    acc["ffn_fused"][0] += 4.0 * R * d * f
                    acc["ffn_fused"][1] += 8.0 * R * d + 2 * 2.0 * f * d
                elif h3 and ffn_fused_h3(d, f):
                    acc["ffn_fused"][0] += 4.0 * R * d * f
                    acc["ffn_fused"][1] += 8.0 * R * d + 2 * 4.0 * f * d
                else:
                    lin(R, d, f, c=h16)
                    lin(R, f, d, a=h16, resadd=True)
            lin(R, d, 3 * hid, c=h16)
            lin(R, hid, d, a=h16, resadd=True)
            for _ in range(2):
                lin(R, d, cfg.value_head_dim * h, c=h16)
                lin(R, cfg.value_head_dim * h, d, a=h16, resadd=True)
                lin(R, d, 2 * d, c=h16)
                lin(R, d, d, a=h16, resadd=True)
    lin(sum((L + 1) // 2 for L in Ls), cfg.max_dim, cfg.joiner_dim)
    return {k: (v[0], v[1]) for k, v in acc.items()}


EPI_NAMES = ["none", "swooshl", "swooshr", "resadd", "mulaux", "mulaux16", "relu", "gelu", "glu"]  # gemm.h


def shape_table(prof: dict, nprof: int, bf16_peak: float, f32_peak: float, nprod: int = 1):
    """Per-shape roofline rows from profile mode 2's "enc_gemm|M|K|N|w16|a16|c16|epi" classes:
    algorithmic bytes (A + W + C [+ C read for EPI_RESADD] at the launch's dtypes) and flops,
    the binding roof (larger of bytes / HBM peak and flops / MFMA peak), and the fraction of
    that roof the measured mean launch time reaches.  nprod > 1 (the split modes): the MFMA
    work is nprod executed bf16 / fp16 products per f32-equivalent one, priced at the dense
    bf16 / fp16 peak (the weight pieces take as many bytes as f32)."""
    rows = []
    for name, (cnt, ms) in prof.items():
        parts = name.split("|")
        if len(parts) != 8:
            continue
        M, K, N, w16, a16, c16, epi = map(int, parts[1:])
        by = (2 if a16 else 4) * M * K + (2 if w16 else 4) * N * K + \
            (2 if c16 else 4) * M * N * (2 if epi == 3 else 1)
        fl = 2.0 * M * K * N * nprod
        t = ms / cnt * 1e-3
        peak_f = bf16_peak if (w16 or nprod > 1) else f32_peak
        t_hbm, t_mfma = by / (HBM_PEAK_GBS * 1e9), fl / (peak_f * 1e12)
        bound = "hbm" if t_hbm >= t_mfma else "mfma"
        rows.append({"M": M, "K": K, "N": N, "a": "bf16" if a16 else "f32",
                     "w": "bf16" if w16 else "f32", "c": "bf16" if c16 else "f32",
                     "epi": EPI_NAMES[epi], "launches_per_step": cnt // nprof,
                     "us": round(t * 1e6, 2), "bytes": by, "flops": fl, "bound": bound,
                     "achieved": round((by / t / 1e9) if bound == "hbm" else (fl / t / 1e12), 1),
                     "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
                     "frac": round(max(t_hbm, t_mfma) / t, 4),
                     "ms_per_step": round(ms / nprof, 4)})
        if nprod > 1:
            rows[-1]["mfma_per_product"] = nprod
    rows.sort(key=lambda r: -r["ms_per_step"])
    return rows


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
    hw = "|hw" if (args.hotwords_file and args.method != "greedy_search") else ""
    key = f"{args.model}|{args.method}|{args.beam if args.method != 'greedy_search' else 1}|" \
          f"{args.precision}|{int(args.audio_sec)}|{kernel_class}{hw}"
    return tab.get(key)


# ------------------------------------------------------------------ CPU baseline
_CPU = {}


def _cpu_worker_init(model, seed, threads, hotwords, variant="greedy-calibrated"):
    import torch
    from oracle.search import HotwordGraph
    from oracle.zipformer import ZipformerOracle
    from zasr.model import PRESETS, variant_weights
    torch.set_num_threads(threads)
    cfg = PRESETS[model]()
    _CPU["orc"] = ZipformerOracle(cfg, variant_weights(cfg, seed, variant))
    _CPU["graph"] = HotwordGraph(*hotwords) if hotwords and hotwords[0] else None


def _cpu_worker_run(job):
    from oracle.fbank import fbank
    from oracle.search import beam_search
    chunks, beam = job
    orc = _CPU["orc"]
    t0 = time.perf_counter()
    for c in chunks:
        enc = orc.encoder(fbank(c))
        beam_search(enc, orc.decoder, orc.joiner, beam, _CPU["graph"] if beam > 1 else None)
    return time.perf_counter() - t0


def cpu_baseline(args, chunks, beam, hotwords, n_chunks=4):
    """The oracle (torch fp32 encoder + numpy fbank + the reference's search restated) on a
    bounded sample, with the reference's CPU policy (BASELINE.md "CPU-baseline plan"):
      * 2 chunk workers when >= 4 chunks and >= 4 physical cores, chunks split even/odd
        (core/asr_engine.py:2262-2276, 2388-2397), one process each;
      * encoder threads = physical cores shared between the workers (:946-955), capped at
        the box's CPU share (16 threads per GPU);
      * 1 warm-up pass then the mean of `--cpu-repeats` timed passes (core/calibration.py:
        822-830).
    Runs before this process touches the GPU (the workers are spawned children)."""
    import multiprocessing as mp
    try:
        import psutil
        phys = psutil.cpu_count(logical=False) or os.cpu_count()
    except Exception:
        phys = os.cpu_count()
    nproc = os.cpu_count()
    share = min(16, phys)
    sample = chunks[:n_chunks]
    workers = 2 if (len(sample) >= 4 and phys >= 4) else 1
    threads = max(1, share // workers)
    jobs = [(sample[w::workers], beam) for w in range(workers)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers, initializer=_cpu_worker_init,
                  initargs=(args.model, WEIGHT_SEED, threads, hotwords, args.weights)) as pool:
        pool.map(_cpu_worker_run, [([c[: SR * 4] for c in j[0][:1]], j[1]) for j in jobs])
        times = []
        for _ in range(max(1, args.cpu_repeats)):
            t0 = time.perf_counter()
            pool.map(_cpu_worker_run, jobs)
            times.append(time.perf_counter() - t0)
    sec = sum(c.shape[0] for c in sample) / SR
    mean = float(np.mean(times))
    return {"value": round(sec / mean, 3), "unit": "audio-sec/sec", "cores": workers * threads,
            "kind": "port", "nproc": nproc, "physical_cores": phys, "workers": workers,
            "threads_per_worker": threads, "repeats": len(times),
            "repeat_s": [round(t, 3) for t in times],
            "sample": f"{len(sample)} planner chunks ({sec:.1f} s) of the benched audio; oracle "
                      f"fbank + torch fp32 encoder + reference search "
                      f"({'greedy' if beam == 1 else 'beam %d' % beam}"
                      f"{' + hotwords' if hotwords and hotwords[0] and beam > 1 else ''}), "
                      f"{workers} worker process(es) x {threads} threads, 1 warm-up + mean of "
                      f"{len(times)}"}


# ------------------------------------------------------------------ CAM++ stage (config 5)
def _campp_cpu(model_seed, feats, threads, repeats):
    import torch
    from oracle.campplus import CamppOracle
    from zasr.campp import CamppConfig, synth_weights
    torch.set_num_threads(threads)
    cfg = CamppConfig()
    orc = CamppOracle(cfg, synth_weights(cfg, model_seed))
    orc.embed(feats[:2])
    times = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        for b in range(0, feats.shape[0], 32):  # the reference's batch (:589-605)
            orc.embed(feats[b:b + 32])
        times.append(time.perf_counter() - t0)
    return float(np.mean(times)), times


def bench_campp(args):
    """CAM++ embeddings of 1 h per GPU: speech regions (the planner's silence-split spans, no
    overlap) -> CAM++ fbank per region -> 150-frame windows every 60 frames (core/speaker_
    diarization_senko_campp_optimized.py:540-582) -> embeddings.  Timed: the embedding of all
    windows (features resident in HBM), `--campp-batch` windows per launch."""
    import torch
    from zasr.binding import CamppEmbedder
    from zasr.campp import CamppConfig, campp_flops, save_model_dir, synth_weights, window_plan
    from zasr.plan import plan_chunks
    from zasr.synth_audio import synth_speech
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    cfg = CamppConfig()
    seed = 20261017
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_bench_campp_{os.getpid()}")
    save_model_dir(mdir, cfg, synth_weights(cfg, seed))
    emb = CamppEmbedder(mdir, device_id=local)
    audio = synth_speech(args.audio_sec, AUDIO_SEED + rank)
    wins = []
    for a, e, _ in plan_chunks(audio, overlap_sec=0.0):
        fb = emb.fbank(audio[a:e])
        wins += [fb[s:s + n] for s, n in window_plan(fb.shape[0]) if n == 150]
    feats = np.ascontiguousarray(np.stack(wins))
    W = feats.shape[0]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = feats[:64]
        mean, times = _campp_cpu(seed, sample, min(16, os.cpu_count() or 1), max(1, args.cpu_repeats))
        cpu = {"value": round(64 / W * args.audio_sec / mean, 3), "unit": "audio-sec/sec",
               "cores": min(16, os.cpu_count() or 1), "kind": "port",
               "repeats": len(times), "sample": f"64 of the {W} windows, oracle CAMPPlus torch fp32, "
                                                 f"batches of 32, 1 warm-up + mean of {len(times)}"}
    d_in = torch.from_numpy(feats).cuda()
    d_out = torch.empty((W, cfg.embedding_size), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    B = max(1, args.campp_batch)

    def step():
        for b in range(0, W, B):
            n = min(B, W - b)
            emb.embed_device(d_in.data_ptr() + b * 150 * 80 * 4, n, 150,
                             d_out.data_ptr() + b * cfg.embedding_size * 4, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
    fl = W * campp_flops(cfg, 150)
    t_step = el / args.steps
    if rank == 0:
        line = {"metric": "audio-sec/sec CAM++ speaker embedding (1.5 s windows, 0.6 s step)",
                "value": round(args.audio_sec * world * args.steps / el, 2),
                "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * t_step, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (seeded speech-like audio, random-init CAM++ weights)",
                "config": {"workload": "CAM++ 192-dim embeddings of 1 h per GPU (config 5 stage)",
                           "windows_per_gpu": W, "launch_batch": B,
                           "windows_per_sec": round(W * world / t_step, 1)},
                "roofline": {"kernel": "campp (whole stage)", "bound": "mfma",
                             "achieved": round(fl / t_step / 1e12, 2),
                             "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(fl / t_step / 1e12 / MFMA_F32_PEAK_TFLOPS, 4),
                             "flops_per_window": campp_flops(cfg, 150)},
                "cpu_baseline": cpu}
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    emb.close()
    if dist:
        dist.destroy_process_group()


# ------------------------------------------------------------------ Silero VAD stage
def _vad_cpu(seed, audio, threads, repeats):
    import torch
    from oracle.silero import SileroOracle, run_windows
    from zasr.silero import SileroConfig, synth_weights
    torch.set_num_threads(threads)
    cfg = SileroConfig()
    sess = SileroOracle(cfg, synth_weights(cfg, seed)).session()
    run_windows(sess, audio[:512 * 50])
    times = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        run_windows(sess, audio)
        times.append(time.perf_counter() - t0)
    return float(np.mean(times)), times


def bench_vad(args):
    """Silero VAD of 1 h per GPU: speech probability of every 512-sample window (64-sample
    context, LSTM state carried; core/vad_utils.py:80-111) with the low-amplitude boost, then
    the host segmentation (get_vad_segments' defaults).  Audio resident in HBM; one step =
    probabilities of the whole hour (`--vad-files` files in one call) + segments."""
    import torch
    from zasr.binding import VadSession
    from zasr.silero import SileroConfig, save_model_dir, synth_weights, window_flops
    from zasr.synth_audio import synth_speech
    from zasr.vad_utils import _segments_from_probs
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    cfg = SileroConfig()
    seed = 20261019
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_bench_vad_{os.getpid()}")
    save_model_dir(mdir, cfg, synth_weights(cfg, seed))
    sess = VadSession(mdir, device_id=local)
    audio = synth_speech(args.audio_sec, AUDIO_SEED + rank)
    F = max(1, args.vad_files)
    bounds = np.linspace(0, len(audio), F + 1).astype(np.int64)
    offs, lens = bounds[:-1], bounds[1:] - bounds[:-1]
    nw = lens // 512
    NW = int(nw.sum())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_s = 512 * 3000
        mean, times = _vad_cpu(seed, audio[:n_s], 1, max(1, args.cpu_repeats))
        cpu = {"value": round(n_s / SR / mean, 2), "unit": "audio-sec/sec", "cores": 1,
               "kind": "port", "repeats": len(times),
               "sample": f"first 3000 windows (96 s) of the hour, the reference's per-window loop "
                         f"(core/vad_utils.py:97-111) over the oracle network, torch fp32 1 thread "
                         f"(the reference's ORT session uses 1 intra-op thread, :30-33); "
                         f"1 warm-up + mean of {len(times)}"}
    d_audio = torch.from_numpy(audio).cuda()
    d_probs = torch.empty(max(1, NW), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    wb = np.concatenate([[0], np.cumsum(nw)])
    segs = []

    def step():
        sess.probs_device(d_audio.data_ptr(), offs, lens, d_probs.data_ptr(), auto_boost=True,
                          stream=stream)
        p = d_probs.cpu().numpy()
        segs.clear()
        for i in range(F):
            segs.append(_segments_from_probs(p[wb[i]:wb[i + 1]], int(lens[i]), SR, 0.2, 100, 250,
                                             1000, 250, True))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
    # the recurrence alone, HIP events on the engine's ordering stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    sess.probs_device(d_audio.data_ptr(), offs, lens, d_probs.data_ptr(), auto_boost=True,
                      stream=stream)
    ev1.record()
    torch.cuda.synchronize()
    t_gpu = ev0.elapsed_time(ev1) / 1e3
    t_step = el / args.steps
    if rank == 0:
        byts = NW * (512 * 4 + 4)  # audio in + probabilities out (the stage's algorithmic bytes)
        line = {"metric": "audio-sec/sec Silero VAD (512-sample windows, segments)",
                "value": round(args.audio_sec * world * args.steps / el, 2),
                "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * t_step, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (seeded speech-like audio, random-init Silero v5 weights)",
                "config": {"workload": f"Silero VAD of {args.audio_sec:.0f} s per GPU as {F} file(s) "
                                       f"(get_vad_segments defaults)",
                           "windows_per_gpu": NW, "files": F,
                           "gpu_ms_probs": round(1000 * t_gpu, 3),
                           "recurrence_passes": sess.last_passes,
                           "n_segments": int(sum(len(x) for x in segs))},
                "roofline": {"kernel": "vad (whole stage: STFT/encoder GEMMs + segmented LSTM)",
                             "bound": "hbm", "achieved": round(byts / t_gpu / 1e9, 2),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(byts / t_gpu / 1e9 / HBM_PEAK_GBS, 5),
                             "traffic": None,
                             "mfma_tflops": round(NW * window_flops(cfg) / t_gpu / 1e12, 3),
                             "note": "the recurrence is latency-bound per step; a file is decoded "
                                     "as ~one segment per CU, parallel in time with verified state "
                                     "continuity (vad.cpp VadEngine::recurrence)"},
                "cpu_baseline": cpu}
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    sess.close()
    if dist:
        dist.destroy_process_group()


# ------------------------------------------------------------------ full pipe (config 5)
def _pipe_cpu_job(job):
    """The config-5 pipe on the CPU oracles for a bounded sample (spawned child: torch thread
    count isolated, no GPU): decode (numpy fbank + torch fp32 encoder + the reference search,
    greedy) of the sample's planner chunks, their words, the merge, CAM++ window embeddings of
    the sample's speech regions (oracle fbank + CAMPPlus, batches of 32 as the reference) and
    the restorer over the sample's transcript (zasr.punct: up to 3 iterations, changed chunks
    re-run, mini-batches of 32) on the ViBERT oracle."""
    import torch
    from oracle.campplus import CamppOracle, campp_fbank
    from oracle.fbank import fbank
    from oracle.search import beam_search
    from oracle.vibert import VibertOracle
    from oracle.zipformer import ZipformerOracle
    from zasr.asr_engine import TokenStats, _words_from_search
    from zasr.campp import CamppConfig, window_plan
    from zasr.campp import synth_weights as campp_weights
    from zasr.merge import merge_chunks_with_overlap
    from zasr.model import PRESETS, synth_tokens, synth_weights
    from zasr.pipeline import make_punctuator, transcript_for_punctuation
    from zasr.vibert import synth_weights as vib_weights
    from zasr.vibert import vibert_base
    model, threads, chunks, offs, regions, repeats = job
    torch.set_num_threads(threads)
    cfg = PRESETS[model]()
    orc = ZipformerOracle(cfg, synth_weights(cfg, WEIGHT_SEED))
    toks = synth_tokens(cfg.vocab_size)
    id2 = dict(enumerate(toks))
    ccfg = CamppConfig()
    corc = CamppOracle(ccfg, campp_weights(ccfg, 20261017))
    vcfg = vibert_base()
    vorc = VibertOracle(vcfg, vib_weights(vcfg, 20261018))

    class Sess:
        def run(self, names, feeds):
            return list(vorc.run(feeds["input_ids"], feeds["attention_mask"],
                                 feeds["token_type_ids"], feeds["input_offsets"]))

    def one_pass():
        per = []
        for c, off in zip(chunks, offs):
            enc = orc.encoder(fbank(c))
            tk, fr, lp, T, emit = beam_search(enc, orc.decoder, orc.joiner, 1)
            per.append({"words": _words_from_search(id2, cfg.vocab_size, len(c), off / SR, tk,
                                                    fr, lp, T, emit),
                        "audio_start_abs": off / SR, "audio_end_abs": (off + len(c)) / SR})
        words, _ = merge_chunks_with_overlap(per)
        wins = []
        for r in regions:
            fb = campp_fbank(r)
            wins += [fb[a:a + n] for a, n in window_plan(fb.shape[0]) if n == 150]
        for b in range(0, len(wins), 32):
            corc.embed(np.stack(wins[b:b + 32]))
        text, hints = transcript_for_punctuation(words)
        make_punctuator(Sess(), vcfg.vocab_size, mini_batch=32).restore(text, pause_hints=hints)
        return len(words), len(wins)

    one_pass()  # warm-up (core/calibration.py:822-830: 1 warm-up, then the mean of repeats)
    times = []
    for _ in range(max(1, repeats)):
        t0 = time.perf_counter()
        nw, nwin = one_pass()
        times.append(time.perf_counter() - t0)
    return times, nw, nwin


def bench_pipe(args):
    """BASELINE config 5 per GPU: one step = one hour through decode (68M, --method,
    --precision) -> word post-processing -> chunk-overlap merge -> ViBERT-capu punctuation of
    the transcript (56-word chunks / 16 overlap, 3 iterations, mini-batches of 32), with the
    CAM++ front end + embeddings of the hour's speech regions (1.5 s windows every 0.6 s) on a
    second stream under the decode, their L2-normalised copy on the host at the end.  The
    audio is resident in HBM; the chunk / region plans are made once (zasr/plan.py)."""
    import torch
    from zasr.binding import CamppEmbedder, Recognizer, VibertSession
    from zasr.campp import CamppConfig, campp_flops
    from zasr.campp import save_model_dir as campp_save
    from zasr.campp import synth_weights as campp_weights
    from zasr.model import PRESETS, chunk_flops, save_model_dir, synth_tokens, synth_weights
    from zasr.pipeline import FullPipe
    from zasr.synth_audio import synth_speech
    from zasr.vibert import save_model_dir as vib_save
    from zasr.vibert import synth_weights as vib_weights
    from zasr.vibert import vibert_base, vibert_flops
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --shard-plan: one hour for the whole job (every rank the same audio, its share of the
    # chunks / regions / ViBERT rows: FullPipe(shard=True)); else each rank its own hour
    audio = synth_speech(args.audio_sec, AUDIO_SEED + (0 if args.shard_plan else rank))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before this process touches the GPU (spawned child); bounded sample: the first two
        # planner chunks and the speech regions they span
        import multiprocessing as mp
        from zasr.plan import plan_chunks
        plan = plan_chunks(audio)[:2]
        end = plan[-1][1]
        regs = [audio[a:e] for a, e, _ in plan_chunks(audio, overlap_sec=0.0) if e <= end]
        threads = min(16, os.cpu_count() or 1)
        with mp.get_context("spawn").Pool(1) as pool:
            times, nw, nwin = pool.map(_pipe_cpu_job, [(args.model, threads,
                                                        [audio[a:e] for a, e, _ in plan],
                                                        [a for a, _, _ in plan], regs,
                                                        args.cpu_repeats)])[0]
        el_cpu = float(np.mean(times))
        cpu = {"value": round(end / SR / el_cpu, 3), "unit": "audio-sec/sec", "cores": threads,
               "kind": "port", "repeats": len(times), "repeat_s": [round(t, 3) for t in times],
               "sample": f"the first {end / SR:.1f} s (2 planner chunks): oracle decode (greedy) "
                         f"+ words + merge, CAM++ oracle on {nwin} windows (batches of 32), the "
                         f"restorer (ViBERT oracle, mini-batches of 32) over {nw} words; torch fp32, "
                         f"{threads} threads, 1 warm-up + mean of {len(times)}"}
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    tmp = tempfile.gettempdir()
    cfg = PRESETS[args.model]()
    beam = 1 if args.method == "greedy_search" else args.beam
    hw_path = DEFAULT_HOTWORDS if args.hotwords_file == "default" else args.hotwords_file
    hotwords = load_hotwords(hw_path, cfg.vocab_size) if (hw_path and beam > 1) else None
    mdir = os.path.join(tmp, f"zasr_pipe_asr_{os.getpid()}")
    toks = synth_tokens(cfg.vocab_size)
    save_model_dir(mdir, cfg, synth_weights(cfg, WEIGHT_SEED), toks)
    rec = Recognizer(mdir, args.method, beam, hotwords=hotwords[0] if hotwords else None,
                     hotword_scores=hotwords[1] if hotwords else None, device_id=local,
                     precision=args.precision)
    recd = {"id2token": dict(enumerate(toks)), "vocab_size": cfg.vocab_size}
    ccfg = CamppConfig()
    cdir = os.path.join(tmp, f"zasr_pipe_campp_{os.getpid()}")
    campp_save(cdir, ccfg, campp_weights(ccfg, 20261017))
    emb = CamppEmbedder(cdir, device_id=local)
    vcfg = vibert_base()
    vdir = os.path.join(tmp, f"zasr_pipe_vibert_{os.getpid()}")
    vib_save(vdir, vcfg, vib_weights(vcfg, 20261018))
    vib = VibertSession(vdir, device_id=local)

    pipe = FullPipe(rec, recd, emb, vib, vcfg.vocab_size, beam=beam, campp_batch=args.campp_batch,
                    shard=args.shard_plan and world > 1)
    pipe.prepare(audio)
    out = {}

    def steps(k):
        # k steps = k passes of the hour through the pipe, pipelined (FullPipe.run_many)
        rs = pipe.run_many(k, args.rover_passes_per_call)
        r = rs[-1]
        out.update(windows=len(r["windows"]), words=len(r["words"]), rows=r["vibert_rows"],
                   vibert_runs=r["vibert_runs"], tokens=r["tokens"],
                   token_ids=[o["token_ids"] for o in rs])

    if args.warmup:
        steps(args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
    t_step = el / args.steps
    # stage times alone (one pass each, serialised): where the step goes
    stage_ms = {}
    main_st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    words, _ = pipe.decode_words(main_st)
    stage_ms["decode_words_merge"] = 1000 * (time.perf_counter() - t1)
    t1 = time.perf_counter()
    pipe.embed_windows(main_st)
    torch.cuda.synchronize()
    stage_ms["campp"] = 1000 * (time.perf_counter() - t1)
    t1 = time.perf_counter()
    s0 = len(pipe.punct.run_shapes)
    pipe.punctuate(words)
    stage_ms["vibert"] = 1000 * (time.perf_counter() - t1)
    vib_shapes = pipe.punct.run_shapes[s0:]
    c_len, plan, regions = pipe.c_len_all, pipe.c_off_all, pipe.r_off_all
    # algorithmic flops of the step: decode + CAM++ windows + ViBERT passes
    f_dec = sum(sum(chunk_flops(cfg, n, beam).values()) for n in c_len)
    f_cam = out["windows"] * campp_flops(ccfg, 150)
    f_vib = sum(vibert_flops(vcfg, B, Lp, Wp) for B, Lp, Wp in vib_shapes)
    fl = f_dec + f_cam + f_vib
    p_dec = MFMA_BF16_PEAK_TFLOPS if args.precision != "fp32" else MFMA_F32_PEAK_TFLOPS
    t_roof = f_dec / (p_dec * 1e12) + (f_cam + f_vib) / (MFMA_F32_PEAK_TFLOPS * 1e12)
    # the decode stage's tokens of every timed pass vs the oracle's decode of the hour (the
    # pipe cuts and weights the bench hour exactly as the config-2 / 3 lines do; data only)
    ocheck = None
    if (world == 1 and not args.shard_plan and
            getattr(args, "weights", "greedy-calibrated") == "greedy-calibrated"):
        chunks_h = [audio[a:a + n] for a, n in zip(pipe.c_off_all, pipe.c_len_all)]
        golden = hour_golden(args, beam, hotwords[0] if hotwords else None, chunks_h)
        if golden is not None:
            ocheck = oracle_agreement(golden[0], golden[1], out["token_ids"], golden[2])
    if rank == 0:
        line = {"metric": "audio-sec/sec full pipe (decode + CAM++ embeddings + ViBERT punctuation)",
                "value": round(args.audio_sec * (1 if args.shard_plan else world) * args.steps / el, 2),
                "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * t_step, 3),
                "higher_is_better": True, "scaling": "strong" if args.shard_plan else "weak",
                "vs_baseline": None,
                "dtype": f"{args.precision} decode, f32 CAM++ / ViBERT",
                "data": "synthetic (seeded speech-like audio, random-init Zipformer / CAM++ / "
                        "ViBERT weights)",
                "config": {"workload": f"BASELINE config 5 per GPU: {args.model} {args.method}"
                                       f"{'' if beam == 1 else ' beam %d' % beam} decode of 1 h "
                                       f"+ merge + CAM++ windows + ViBERT-capu punctuation",
                           "decode_chunks": len(plan), "campp_regions": len(regions),
                           "parallelism": (f"dp{world} (one hour for the job: each rank its LPT "
                                           f"share of the chunks and regions and of every ViBERT "
                                           f"run's rows; words / embeddings / logits gathered to "
                                           f"every rank by host object gathers; strong scaling)"
                                           if args.shard_plan else
                                           f"dp{world} (each rank its own hour; weak scaling)"),
                           "shard_chunks_this_rank": len(pipe.c_len) if args.shard_plan else None,
                           "campp_windows": out["windows"], "campp_launch_batch": args.campp_batch,
                           "words": out["words"], "tokens": out["tokens"],
                           "vibert_rows_per_iteration": out["rows"],
                           "vibert_runs_per_step": out["vibert_runs"],
                           "vibert_iterations": "the reference's restorer (zasr.punct): edits "
                                                "applied, later iterations re-run only the "
                                                "chunks whose text changed; one run per "
                                                "iteration (bit-identical to its 32-row "
                                                "mini-batches, tests/test_gpu_pipe.py)",
                           "stage_ms_alone": {k: round(v, 2) for k, v in stage_ms.items()}},
                "roofline": {"kernel": "whole pipe (algorithmic flops / step time)",
                             "bound": "mfma", "unit": "TFLOP/s",
                             "achieved": round(fl / t_step / 1e12, 2),
                             "peak": round(fl / t_roof / 1e12, 2),
                             "frac": round(t_roof / t_step, 4),
                             "flops_per_step": {"decode": f_dec, "campp": f_cam, "vibert": f_vib},
                             "note": "peak = the mixed roof: decode flops at the bf16 MFMA peak "
                                     "(f32 in fp32 mode) + CAM++ / ViBERT flops at the f32 MFMA "
                                     "peak (exact f32, their reference tolerances); per-stage "
                                     "roofs in the asr / campp stage lines"},
                "cpu_baseline": cpu}
        if ocheck is not None:
            line["oracle_check"] = ocheck
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    rec.close()
    emb.close()
    vib.close()
    if dist:
        dist.destroy_process_group()


# ------------------------------------------------------------------ ROVER pair (config 4)
def _rover_cpu_job(job):
    """Config 4 on the CPU oracles for a bounded sample (spawned child, no GPU): both models'
    oracle decode (numpy fbank once per chunk, shared as the reference does; torch fp32
    encoders; the reference search, beam + hotword graph), their words and the block vote."""
    import torch
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from oracle.zipformer import ZipformerOracle
    from zasr.asr_engine import _words_from_search
    from zasr.model import PRESETS, synth_tokens, synth_weights
    from zasr.rover import rover_merge
    threads, chunks, offs, beam, hw_path, phrases, repeats = job
    torch.set_num_threads(threads)
    models = []
    for name, seed in (("zipformer-30m", WEIGHT_SEED + 1), ("zipformer-68m", WEIGHT_SEED)):
        cfg = PRESETS[name]()
        hw = load_hotwords(hw_path, cfg.vocab_size) if hw_path else None
        models.append((cfg, ZipformerOracle(cfg, synth_weights(cfg, seed)),
                       dict(enumerate(synth_tokens(cfg.vocab_size))),
                       HotwordGraph(*hw) if hw and hw[0] else None))
    def one_pass():
        n_words = 0
        for c, off in zip(chunks, offs):
            f = fbank(c)
            per = []
            for cfg, orc, id2, graph in models:
                tk, fr, lp, T, emit = beam_search(orc.encoder(f), orc.decoder, orc.joiner, beam,
                                                  graph)
                per.append(_words_from_search(id2, cfg.vocab_size, len(c), off / SR, tk, fr, lp,
                                              T, emit))
            n_words += len(rover_merge(per[0], per[1], phrases)[0])
        return n_words

    one_pass()  # warm-up (core/calibration.py:822-830: 1 warm-up, then the mean of repeats)
    times = []
    for _ in range(max(1, repeats)):
        t0 = time.perf_counter()
        n_words = one_pass()
        times.append(time.perf_counter() - t0)
    return times, n_words


def bench_rover(args):
    """BASELINE config 4 per GPU: one step = the hour's planner chunks through Zipformer-30M
    (primary) and Zipformer-68M, both modified beam search with beam --beam (the reference's
    decode_chunk always runs _ort_beam_search with max_active_paths = 8,
    core/asr_engine.py:1224, :2041-2044), concurrently on the GPU, then the per-chunk block vote
    and the chunk-overlap merge on the host, pipelined with the next step's decode
    (zasr.rover.rover_device_many).  Audio resident in HBM."""
    import torch
    from zasr.binding import Recognizer
    from zasr.model import PRESETS, chunk_flops, save_model_dir, synth_tokens, synth_weights
    from zasr.rover import rover_device_many
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    beam = args.beam
    # --shard-plan: one hour for the whole job, each rank decodes + votes its LPT share of the
    # chunks and the voted chunks are gathered in chunk order for the merge (zasr.rover)
    chunks = make_chunks(args.audio_sec, AUDIO_SEED + (0 if args.shard_plan else rank))
    lens = [c.shape[0] for c in chunks]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    mine = None
    if args.shard_plan:
        mine = shard_share(lens, world, rank, args.proxy_ranks)
    hw_path = (DEFAULT_HOTWORDS if args.hotwords_file == "default" else args.hotwords_file) or ""
    phrases = []
    if hw_path:
        from zasr.hotword_context import parse_hotwords_file
        phrases = [p for p, _ in parse_hotwords_file(hw_path, 1.5)]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before this process touches the GPU (spawned child); bounded sample: the first chunk
        import multiprocessing as mp
        threads = min(16, os.cpu_count() or 1)
        with mp.get_context("spawn").Pool(1) as pool:
            times, nw = pool.map(_rover_cpu_job, [(threads, chunks[:1], offs[:1], beam, hw_path,
                                                   phrases, args.cpu_repeats)])[0]
        el_cpu = float(np.mean(times))
        cpu = {"value": round(lens[0] / SR / el_cpu, 3), "unit": "audio-sec/sec",
               "cores": threads, "kind": "port", "repeats": len(times),
               "repeat_s": [round(t, 3) for t in times],
               "sample": f"the first planner chunk ({lens[0] / SR:.1f} s): oracle fbank once, "
                         f"30M and 68M torch fp32 encoders + the reference search (beam {beam}"
                         f"{' + hotwords' if phrases else ''}), words, block vote ({nw} words); "
                         f"{threads} threads, 1 warm-up + mean of {len(times)}"}
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    recs, recds, cfgs = [], [], []
    for name, seed in (("zipformer-30m", WEIGHT_SEED + 1), ("zipformer-68m", WEIGHT_SEED)):
        cfg = PRESETS[name]()
        hotwords = load_hotwords(hw_path, cfg.vocab_size) if hw_path else None
        mdir = os.path.join(tempfile.gettempdir(), f"zasr_rover_{name}_{os.getpid()}")
        toks = synth_tokens(cfg.vocab_size)
        save_model_dir(mdir, cfg, synth_weights(cfg, seed), toks)
        recs.append(Recognizer(mdir, "modified_beam_search", beam,
                               hotwords=hotwords[0] if hotwords else None,
                               hotword_scores=hotwords[1] if hotwords else None,
                               device_id=local, precision=args.precision))
        recds.append({"id2token": dict(enumerate(toks)), "vocab_size": cfg.vocab_size})
        cfgs.append(cfg)
    d_wav = torch.from_numpy(np.concatenate(chunks)).cuda()
    torch.cuda.synchronize()
    last = {}
    toks = []  # per timed pass: (30M token ids per chunk, 68M token ids per chunk)

    def steps(k, keep=False):
        r = rover_device_many(recs[0], recs[1], recds[0], recds[1], d_wav.data_ptr(), offs, lens,
                              k, beam, phrases, args.rover_sub_batches,
                              args.rover_passes_per_call, mine=mine,
                              gather=not (args.proxy_ranks > 1 and world == 1),
                              tokens_out=toks if keep else None)[-1]
        last.update(words=len(r[0]), disagree_blocks=sum(r[1]), tokens_a=r[2], tokens_b=r[3])

    if args.warmup:
        steps(args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps, keep=mine is None and rank == 0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
    # both models' tokens of every timed pass against the oracle's decode of this hour
    # (tests/golden/bench_hour_oracle_rover.json, make_bench_hour_golden.py --set rover)
    ochecks = rover_golden_checks(args, beam, phrases, chunks, toks) if toks else None
    # each model alone (decode only, HIP work + result copies) for the breakdown
    alone = {}
    sel = list(range(len(lens))) if mine is None else mine
    for name, rec in zip(("30m", "68m"), recs):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if sel:
            rec.decode_device(d_wav.data_ptr(), [offs[i] for i in sel], [lens[i] for i in sel],
                              beam=beam)
        alone[name] = round(1000 * (time.perf_counter() - t1), 2)
    t_step = el / args.steps
    fl = sum(sum(chunk_flops(c, n, beam).values()) for c in cfgs for n in lens)
    peak = MFMA_BF16_PEAK_TFLOPS if args.precision != "fp32" else MFMA_F32_PEAK_TFLOPS
    if rank == 0:
        line = {"metric": "audio-sec/sec (xRT) ROVER Zipformer-30M + 68M offline decode",
                "value": round(args.audio_sec * (1 if args.shard_plan else world) * args.steps / el, 2),
                "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * t_step, 3),
                "higher_is_better": True, "scaling": "strong" if args.shard_plan else "weak",
                "vs_baseline": None,
                "dtype": args.precision,
                "data": "synthetic (seeded speech-like audio, random-init Zipformer-30M / 68M weights)",
                "config": {"workload": f"BASELINE config 4 per GPU: zipformer-30m + zipformer-68m "
                                       f"modified_beam_search beam {beam}"
                                       f"{' + hotwords' if phrases else ''}, 1 h of planner "
                                       f"chunks, block vote + overlap merge",
                           "chunks_per_gpu": len(lens), "sub_batches": args.rover_sub_batches,
                           "passes_per_call": args.rover_passes_per_call,
                           "words": last["words"],
                           "disagreeing_blocks": last["disagree_blocks"],
                           "tokens_30m": last["tokens_a"], "tokens_68m": last["tokens_b"],
                           "decode_alone_ms": alone,
                           "shard_chunks_this_rank": len(mine) if mine is not None else None,
                           "proxy_ranks": args.proxy_ranks or None,
                           "parallelism": (f"dp{world} (one hour for the job: each rank decodes "
                                           f"and votes its LPT share of the chunks, the voted "
                                           f"chunks gathered to every rank in chunk order by a "
                                           f"host object gather, merged there; strong scaling)"
                                           if args.shard_plan else
                                           f"dp{world} (each rank its own hour; weak scaling)")},
                "oracle_check": ochecks,
                "token_exact": (all(c["chunks_identical_to_oracle"].split("/")[0] ==
                                    c["chunks_identical_to_oracle"].split("/")[1] or
                                    bool(c["differing_chunks_all_audited_f32_ties"])
                                    for c in ochecks.values()) if ochecks else None),
                "roofline": {"kernel": "both encoders + joiners (algorithmic flops / step time)",
                             "bound": "mfma", "unit": "TFLOP/s",
                             "achieved": round(fl / t_step / 1e12, 2), "peak": peak,
                             "frac": round(fl / t_step / 1e12 / peak, 4),
                             "flops_per_step": fl},
                "cpu_baseline": cpu}
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    for r in recs:
        r.close()
    if dist:
        dist.destroy_process_group()


# ------------------------------------------------------------------ strong scaling
def gather_shards(res, mine, n_all, k, dist, partial=False):
    """--shard-plan: every rank's results of its LPT share over k pipelined steps -> the last
    step's results of ALL chunks, in chunk order, on every rank (host object gather, the
    decode_sharded protocol of zasr.shard; no collective on the GPU data path).  The payload
    is what a caller needs per chunk: token ids, frames, log-probs, stats, T'."""
    n = len(mine)
    part = []
    for s in range(k):
        for j, i in enumerate(mine):
            r = res[s * n + j]
            part.append((s, i, {a: getattr(r, a) for a in ("token_ids", "frames", "log_probs",
                                                              "stats", "T") if hasattr(r, a)}))
    parts = [part]
    if dist:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, part)
    from types import SimpleNamespace
    out = [None] * n_all
    for p in parts:
        for s, i, d in p:
            if s == k - 1:
                out[i] = SimpleNamespace(**d)
    if partial:  # --proxy-ranks: only this share was decoded
        return [r for r in out if r is not None]
    missing = [i for i, r in enumerate(out) if r is None]
    if missing:
        raise RuntimeError(f"shard gather lost chunks {missing[:5]}")
    return out


# ------------------------------------------------------------------ token-exact mode
SPLIT_PRODUCTS = {"bf16x3": 3, "bf16x6": 6, "f16x3": 3}


def parity_mode_line(args, cfg, mdir, hotwords, beam, d_wav, offs, lens, stream, fl_step,
                     L_list, dist, dev, golden=None):
    """The same workload (same audio in HBM, same batched pipeline, same step count semantics)
    in the token-exact precision mode: xRT, ms per step, the end-to-end roofline against the
    f32 MFMA peak (the precision the mode reproduces) and, for the split-bf16 modes, the
    fraction of the bf16 MFMA peak their split products occupy; the dominant kernel class's
    roofline from the library's HIP-event class profile."""
    import torch
    from zasr.binding import Recognizer
    prec = args.parity_precision
    rec = Recognizer(mdir, args.method, beam, hotwords=hotwords[0] if hotwords else None,
                     hotword_scores=hotwords[1] if hotwords else None,
                     device_id=int(os.environ.get("LOCAL_RANK", "0")), precision=prec)
    n = len(lens)
    k = max(1, args.parity_steps or args.steps)

    def steps(m):
        return rec.decode_device_batches(d_wav.data_ptr(), offs * m, lens * m, [n] * m,
                                         beam=beam, stream=stream)

    first = steps(1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = steps(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the claim, measured: the timed batches' tokens against an exact-f32 decode of the same
    # chunks (the fp32 mode: exact-f32 MFMA, f64 FFT; tests pin it token-exact to the oracle)
    check = None
    if not args.no_parity_check and prec != "fp32":
        ref_rec = Recognizer(mdir, args.method, beam, hotwords=hotwords[0] if hotwords else None,
                             hotword_scores=hotwords[1] if hotwords else None,
                             device_id=int(os.environ.get("LOCAL_RANK", "0")), precision="fp32")
        ref = ref_rec.decode_device(d_wav.data_ptr(), offs, lens, beam=beam, stream=stream)
        torch.cuda.synchronize()
        ref_rec.close()
        ref_toks = [r.token_ids.tolist() for r in ref]
        steps_same = []
        for st in range(k):
            got = [r.token_ids.tolist() for r in res[st * n:(st + 1) * n]]
            steps_same.append(sum(a == b for a, b in zip(got, ref_toks)))
        diff = [i for i, (a, b) in enumerate(zip([r.token_ids.tolist() for r in res[-n:]], ref_toks))
                if a != b]
        lp_max = max((float(np.max(np.abs(a.log_probs - b.log_probs)))
                      for a, b in zip(res[-n:], ref) if a.token_ids.tolist() == b.token_ids.tolist()
                      and a.log_probs.size), default=0.0)
        check = {"chunks_identical_to_fp32": f"{min(steps_same)}/{n}",
                 "per_timed_step": steps_same,
                 "fp32_tokens": int(sum(len(t) for t in ref_toks)),
                 "differing_chunks": diff[:20],
                 "max_abs_log_prob_diff_identical_chunks": lp_max,
                 "reference": "the same chunks decoded by the fp32 mode (exact-f32 MFMA), "
                              "same search"}
    ocheck = None
    if golden is not None:
        ocheck = oracle_agreement(golden[0], golden[1],
                                  [[r.token_ids.tolist() for r in res[st * n:(st + 1) * n]]
                                   for st in range(k)], golden[2])
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=dev)
    rec.profile(1)
    rec.profile_reset()
    rec.decode_device(d_wav.data_ptr(), offs, lens, beam=beam, stream=stream)
    torch.cuda.synchronize()
    classes = rec.profile_report()
    rec.profile(0)
    rec.close()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    t_step = el / k
    f32_tf = fl_step / t_step / 1e12
    # roofline fractions are against the peak of the MFMA the mode EXECUTES: the split modes
    # run SPLIT_PRODUCTS[prec] fp16 / bf16 MFMAs per f32-equivalent product (dense 2.5 PF),
    # fp32 runs the f32-input MFMA (157.3 TF)
    nprod = SPLIT_PRODUCTS.get(prec, 1)
    peak_exec = MFMA_BF16_PEAK_TFLOPS if prec in SPLIT_PRODUCTS else MFMA_F32_PEAK_TFLOPS
    mfma_exec = {"bf16x3": "bf16", "bf16x6": "bf16", "f16x3": "fp16"}.get(prec, "f32")
    out = {"precision": prec, "value": round(args.audio_sec * world * k / el, 2),
           "unit": "audio-sec/sec", "steps": k, "ms_per_step": round(1000 * t_step, 3),
           "oracle_check": ocheck,
           "parity_check": check,
           # identical to the oracle on every chunk except audited f32 ties (the GPU fp32
           # mode differs from the oracle on exactly those chunks too: parity_check)
           "token_exact": ((ocheck["chunks_identical_to_oracle"] == f"{n}/{n}" or
                            bool(ocheck["differing_chunks_all_audited_f32_ties"])) if ocheck else
                           (check["chunks_identical_to_fp32"] == f"{n}/{n}") if check else None),
           "parity_evidence": "oracle_check (every timed batch vs the oracle's decode of this hour, "
                              "tests/golden/bench_hour_oracle.json), parity_check (vs the GPU fp32 "
                              "mode, same run) and tests/test_gpu_hour.py",
           "roofline_e2e": {"flops_per_step": fl_step, "f32_equivalent_tflops": round(f32_tf, 2),
                            "executed_mfma": mfma_exec, "mfma_per_product": nprod,
                            "achieved": round(nprod * f32_tf, 2), "unit": "TFLOP/s",
                            "peak": peak_exec,
                            "frac": round(nprod * f32_tf / peak_exec, 4)},
           "kernel_classes_ms_per_step": {kk: round(v[1], 3) for kk, v in classes.items()}}
    if classes:
        dom, (cnt, ms) = max(classes.items(), key=lambda kv: kv[1][1])
        per = ms / cnt * 1e-3
        if dom in ("enc_gemm", "ffn_fused"):
            f_cls = gemm_class_work(cfg, L_list, False, h3=prec == "f16x3")[dom][0]
            tf = f_cls / cnt / per / 1e12
            out["roofline"] = {"kernel": dom, "bound": "mfma", "avg_launch_ms": round(per * 1e3, 4),
                               "launches_per_step": cnt, "f32_equivalent_tflops": round(tf, 2),
                               "executed_mfma": mfma_exec, "mfma_per_product": nprod,
                               "achieved": round(nprod * tf, 2), "unit": "TFLOP/s",
                               "peak": peak_exec, "frac": round(nprod * tf / peak_exec, 4)}
        else:
            out["roofline"] = {"kernel": dom, "avg_launch_ms": round(per * 1e3, 4),
                               "launches_per_step": cnt}
    return out


# ------------------------------------------------------------------ drop-in loop
def bench_dropin(args):
    """The reference's transcription phase restated over the drop-in surface: the planner
    (find_silent_regions -> ~30 s chunks with 3 s overlap, core/asr_engine.py:2137-2161; the
    zasr.dropin hook registers the plan), TWO worker threads calling decode_chunk per chunk on
    even / odd indices (:2326-2397; the recognizer of the reference's decode_chunk is always
    modified beam search with max_active_paths, :1224), the timestamp map and the chunk-overlap
    merge (:2488-2494).  One step = the whole phase for 1 h of host-resident audio (the
    reference's waveform is a numpy array), hotwords per --hotwords-file.  The plan-ahead route
    makes the two workers' 121 calls ONE batched GPU decode; --no-pipeline sets
    ZASR_PLAN_AHEAD=0 (every call its own decode, the round-2 behaviour)."""
    if args.no_pipeline:
        os.environ["ZASR_PLAN_AHEAD"] = "0"
    import threading

    import torch
    from zasr import asr_engine as ae
    from zasr.merge import merge_chunks_with_overlap
    from zasr.model import PRESETS, save_model_dir, synth_tokens, variant_weights
    from zasr.plan import best_split, concat_to_original, silent_regions
    from zasr.synth_audio import synth_speech
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    cfg = PRESETS[args.model]()
    beam = args.beam
    hw_path = DEFAULT_HOTWORDS if args.hotwords_file == "default" else args.hotwords_file
    hotwords = load_hotwords(hw_path, cfg.vocab_size) if hw_path else ([], [])
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_dropin_{args.model}_{os.getpid()}")
    save_model_dir(mdir, cfg, variant_weights(cfg, WEIGHT_SEED, args.weights),
                   synth_tokens(cfg.vocab_size))
    # the drop-in's own default precision (zasr.asr_engine.DEFAULT_PRECISION: what install()
    # users get) unless --precision is given explicitly
    prec = args.precision if any(a.startswith("--precision") for a in sys.argv[1:]) \
        else ae.DEFAULT_PRECISION
    rec = ae.create_recognizer(mdir, 4, max_active_paths=beam, hotwords=hotwords,
                               device_id=local, precision=prec)
    concat = synth_speech(args.audio_sec, AUDIO_SEED + rank)
    omap = [(0, 0, len(concat))]  # no VAD cut: the identity offset map (:2181)
    info = {}

    split = {"regions": 0.0, "decode_start": 0.0, "decode": 0.0, "after_decode": 0.0, "merge": 0.0}

    def phase():
        # the planner (:2137-2161) through the hook the drop-in installs on find_silent_regions:
        # the GPU silence detector (the signal stays in HBM, the plan's decode starts at once),
        # or with --no-pipeline / ZASR_GPU_PLANNER=0 the reference's numpy function
        t0 = time.perf_counter()
        regions = ae.plan_ahead_regions(concat, best_split)
        if regions is None:
            regions = silent_regions(concat)
            ae.register_plan_from_regions(concat, regions, best_split)
        from zasr.plan import plan_from_regions
        plan = plan_from_regions(len(concat), regions, best_split)
        results = [None] * len(plan)

        def worker(idx):
            for i in idx:
                s, e, ov = plan[i]
                words = ae.decode_chunk(rec, concat[s:e], s / SR)
                for w in words:
                    w["start"] = concat_to_original(w["start"], omap)
                    w["end"] = concat_to_original(w["end"], omap)
                results[i] = {"words": words, "audio_start_abs": s / SR, "audio_end_abs": e / SR,
                              "overlap_sec": ov / SR}

        ts = [threading.Thread(target=worker, args=(list(range(k, len(plan), 2)),))
              for k in (0, 1)]
        t1 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        t2 = time.perf_counter()
        merged, _ = merge_chunks_with_overlap(results)
        t3 = time.perf_counter()
        info.update(chunks=len(plan), words=len(merged))
        # phase split (ms per step, summed over the timed steps): the planner call, the plan's
        # background decode, the workers' word building after it, the merge
        jobs = [j for sig in ae._planned[-1:] for per in sig.jobs.values() for j in per.values()]
        dec = jobs[0] if jobs and jobs[0].t_end is not None else None
        split["regions"] += t1 - t0
        split["decode_start"] += (dec.t_start - t0) if dec else 0.0
        split["decode"] += (dec.t_end - dec.t_start) if dec else 0.0
        split["after_decode"] += (t2 - max(dec.t_end, t1)) if dec else t2 - t1
        split["merge"] += t3 - t2

    for _ in range(args.warmup):
        phase()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    for k in split:
        split[k] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        phase()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=f"cuda:{local}")
    if rank == 0:
        line = {"metric": "audio-sec/sec (xRT) drop-in decode_chunk loop (reference two-worker "
                          "dispatch), Zipformer-68M",
                "value": round(args.audio_sec * world * args.steps / el, 2),
                "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": prec,
                "data": "synthetic (seeded speech-like audio, random-init Zipformer weights)",
                "config": {"workload": f"{args.model} modified_beam_search beam {beam}"
                                       f"{' + hotwords' if hotwords[0] else ''} through "
                                       f"zasr.asr_engine.decode_chunk from two worker threads, "
                                       f"1 h of host audio per GPU, timestamps mapped, overlap merge",
                           "plan_ahead": os.environ.get("ZASR_PLAN_AHEAD", "1") != "0",
                           "gpu_planner": ae._gpu_planner_on(),
                           "phase_ms_per_step": {k: round(1000 * v / args.steps, 3)
                                                 for k, v in split.items()},
                           **info},
                "roofline": None, "cpu_baseline": None}
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    ae.clear_model_cache()
    if dist:
        dist.destroy_process_group()


# ------------------------------------------------------------------ main
def run_parity_child():
    """The parity-mode line measured in a CHILD process (this process has initialised the
    GPU: the child is started, never exec'd into).  A second engine in this process would put
    its streams on hardware queues the headline engine already holds (streams beyond
    GPU_MAX_HW_QUEUES share queues in creation order and serialise): the mode
    measured 26k xRT beside the headline engine vs its own pipeline's rate alone."""
    cmd = [sys.executable, os.path.abspath(__file__), "--parity-child"] + sys.argv[1:]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
    for line in r.stdout.splitlines():
        if line.startswith("PARITY_JSON "):
            return json.loads(line[len("PARITY_JSON "):])
    sys.stderr.write(r.stdout[-2000:] + r.stderr[-4000:])
    raise RuntimeError(f"parity-mode child failed (rc {r.returncode})")


def run_sub_bench(argv, timeout=900):
    """Another bench.py workload in a CHILD process (own HIP context and hardware queues; this
    process has initialised the GPU, so it starts a child and never execs): its JSON line."""
    cmd = [sys.executable, os.path.abspath(__file__)] + argv
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    for line in reversed(r.stdout.splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    sys.stderr.write(r.stdout[-2000:] + r.stderr[-4000:])
    raise RuntimeError(f"sub-bench {' '.join(argv)} failed (rc {r.returncode})")


def sub_line(d):
    """The fields of a child bench line the parent carries."""
    keep = ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config",
            "oracle_check", "token_exact", "roofline", "kernel_classes_ms_per_step")
    out = {k: d[k] for k in keep if k in d}
    if "config" in out:
        out["config"] = {k: v for k, v in out["config"].items()
                         if k in ("workload", "weights", "single_batch_latency_ms",
                                  "emitting_frame_fraction", "tokens_30m", "tokens_68m",
                                  "decode_alone_ms")}
    if out.get("oracle_check") and "token_exact" not in out:
        oc = out["oracle_check"]
        n = oc["chunks_identical_to_oracle"].split("/")
        out["token_exact"] = n[0] == n[1] or bool(oc["differing_chunks_all_audited_f32_ties"])
    return out


def parity_child_main(args):
    """--parity-child: the bench workload (same chunks, same weights) in the parity precision
    only; prints one PARITY_JSON line for the parent (run_parity_child)."""
    import torch
    from zasr.model import PRESETS, chunk_flops, save_model_dir, synth_tokens, variant_weights
    cfg = PRESETS[args.model]()
    beam = 1 if args.method == "greedy_search" else args.beam
    hw_path = DEFAULT_HOTWORDS if args.hotwords_file == "default" else args.hotwords_file
    hotwords = load_hotwords(hw_path, cfg.vocab_size) if (hw_path and beam > 1) else None
    chunks = make_chunks(args.audio_sec, AUDIO_SEED)
    lens = [c.shape[0] for c in chunks]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    torch.cuda.set_device(0)
    dev = "cuda:0"
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_parity_{args.model}_{os.getpid()}")
    save_model_dir(mdir, cfg, variant_weights(cfg, WEIGHT_SEED, args.weights),
                   synth_tokens(cfg.vocab_size))
    d_wav = torch.from_numpy(np.concatenate(chunks)).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    fl_step = sum(sum(chunk_flops(cfg, n, beam).values()) for n in lens)
    L_list = [((n + 80) // 160 - 7) // 2 for n in lens]
    out = parity_mode_line(args, cfg, mdir, hotwords, beam, d_wav, offs, lens, stream, fl_step,
                           L_list, None, dev, golden=hour_golden(args, beam, hotwords, chunks))
    out["process"] = "child of the bench process (own HIP context and hardware queues)"
    print("PARITY_JSON " + json.dumps(out), flush=True)


def main():
    args = parse_args()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.parity_child:
        return parity_child_main(args)
    if args.stage == "campp":
        return bench_campp(args)
    if args.stage == "vad":
        return bench_vad(args)
    if args.stage == "pipe":
        return bench_pipe(args)
    if args.stage == "rover":
        return bench_rover(args)
    if args.stage == "dropin":
        return bench_dropin(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    from zasr.model import PRESETS, chunk_flops
    cfg = PRESETS[args.model]()
    beam = 1 if args.method == "greedy_search" else args.beam
    hw_path = DEFAULT_HOTWORDS if args.hotwords_file == "default" else args.hotwords_file
    hotwords = load_hotwords(hw_path, cfg.vocab_size) if (hw_path and beam > 1) else None

    # each rank: its own hour of audio (weak scaling), planned like the reference; with
    # --shard-plan one hour for the whole job, each rank its LPT share of the chunks
    all_chunks = make_chunks(args.audio_sec, AUDIO_SEED + (0 if args.shard_plan else rank))
    if args.shard_plan:
        mine = shard_share([c.shape[0] for c in all_chunks], world, rank, args.proxy_ranks)
    else:
        mine = list(range(len(all_chunks)))
    chunks = [all_chunks[i] for i in mine]
    lens = [c.shape[0] for c in chunks]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.cpu_dry_run:
        cpu = cpu_baseline(args, chunks, beam, hotwords)

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo" if args.cpu_dry_run else "nccl", init_method="env://")

    rec, dev = None, None
    if args.cpu_dry_run:
        # launcher / rank / timing path only: a CPU stand-in for the decode (one small result
        # per chunk, so the --shard-plan gather moves real objects)
        from types import SimpleNamespace

        def steps(k):
            out = []
            for _ in range(k):
                out += [SimpleNamespace(token_ids=np.arange(int(np.abs(c[::97]).sum()) % 7 + 1),
                                        T=c.shape[0] // 640) for c in chunks]
            return out if args.shard_plan else out[len(out) - len(chunks):]
    else:
        torch.cuda.set_device(local)
        dev = f"cuda:{local}"
        from zasr.binding import Recognizer
        from zasr.model import save_model_dir, synth_tokens, variant_weights
        weights = variant_weights(cfg, WEIGHT_SEED, args.weights)
        mdir = os.path.join(tempfile.gettempdir(), f"zasr_bench_{args.model}_{os.getpid()}")
        save_model_dir(mdir, cfg, weights, synth_tokens(cfg.vocab_size))
        del weights
        rec = Recognizer(mdir, args.method, beam, hotwords=hotwords[0] if hotwords else None,
                         hotword_scores=hotwords[1] if hotwords else None, device_id=local,
                         precision=args.precision)
        offs = np.cumsum([0] + lens[:-1]).tolist()
        d_wav = torch.from_numpy(np.concatenate(chunks) if chunks else np.zeros(1, np.float32)).to(dev)
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
            if n == 0:  # --shard-plan with more ranks than chunks
                return []
            r = rec.decode_device_batches(d_wav.data_ptr(), offs * k, lens * k, [n] * k,
                                          beam=beam, stream=stream)
            return r if args.shard_plan else r[-n:]

    def sync():
        if dev is not None:
            torch.cuda.synchronize()

    if args.warmup:
        steps(args.warmup)
    sync()
    batch_latency_ms = None
    if rec is not None:  # one batch alone (nothing to overlap with): reported beside
        t1 = time.perf_counter()
        step()
        sync()
        batch_latency_ms = 1000 * (time.perf_counter() - t1)

    # timed region: barrier + sync on both sides, max over ranks
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    res = steps(args.steps)
    sync()
    if args.shard_plan:
        res = gather_shards(res, mine, len(all_chunks), args.steps, dist,
                            partial=args.proxy_ranks > 1 and not dist)
    el = time.perf_counter() - t0
    if dist:
        from zasr.shard import max_over_ranks
        el = max_over_ranks(el, device=dev)
        dist.barrier()

    # kernel-class timing: HIP events recorded by the library on its launch stream over
    # profiled steps (separate from the wall-clock region above)
    classes, shapes, nprof = {}, None, max(1, min(args.steps, 3))
    if rec is not None:
        rec.profile(1)
        rec.profile_reset()
        for _ in range(nprof):
            step()
        sync()
        classes = rec.profile_report()
        if args.shape_table:
            rec.profile(2)
            rec.profile_reset()
            step()
            sync()
            shapes = shape_table(rec.profile_report(), 1, MFMA_BF16_PEAK_TFLOPS,
                                 MFMA_F32_PEAK_TFLOPS, SPLIT_PRODUCTS.get(args.precision, 1))
        rec.profile(0)

    # weak: every rank its own hour; strong (--shard-plan): one hour for the whole job
    value = args.audio_sec * (1 if args.shard_plan else world) * args.steps / el
    emitted = sum(int(r.token_ids.size) for r in res)
    tprime = sum(int(r.T) for r in res)

    L_list = [((n + 80) // 160 - 7) // 2 for n in lens]
    bf16 = args.precision != "fp32"
    peak_mfma = MFMA_BF16_PEAK_TFLOPS if bf16 else MFMA_F32_PEAK_TFLOPS
    # end-to-end roofline: algorithmic FLOPs of the whole path per step
    # (zasr.model.chunk_flops over the step's chunks) / step time / MFMA peak
    fl_parts = {}
    for n in lens:
        for k, v in chunk_flops(cfg, n, beam).items():
            fl_parts[k] = fl_parts.get(k, 0.0) + v
    fl_step = sum(fl_parts.values())
    t_step = el / args.steps
    e2e = {"flops_per_step": fl_step, "flops_per_audio_sec": round(fl_step / args.audio_sec),
           "breakdown_gflop_per_step": {k: round(v / 1e9, 2) for k, v in fl_parts.items()},
           "achieved": round(fl_step / t_step / 1e12, 2), "unit": "TFLOP/s", "peak": peak_mfma,
           "frac": round(fl_step / t_step / 1e12 / peak_mfma, 4)}

    # bf16 / bf16_enc store the GEMM intermediates in bf16; the split modes in f32 (their MFMA
    # work is nprod executed products per f32-equivalent one)
    work = gemm_class_work(cfg, L_list, args.precision in ("bf16", "bf16_enc"),
                           h3=args.precision == "f16x3")
    nprod = SPLIT_PRODUCTS.get(args.precision, 1)
    f_join = 2.0 * beam * tprime * cfg.joiner_dim * cfg.vocab_size  # per step
    dom = max(classes.items(), key=lambda kv: kv[1][1])[0] if classes else None
    roof = None
    if dom:
        cnt, ms = classes[dom]
        per_launch_s = ms / cnt * 1e-3
        if dom in work:
            # the binding roof is the larger of bytes / HBM peak and flops / MFMA peak
            f_cls, b_cls = work[dom]
            fl, by = nprod * f_cls * nprof / cnt, b_cls * nprof / cnt  # per launch (class mean)
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
                if nprod > 1:  # executed MFMA flops: nprod products per f32-equivalent one
                    roof["mfma_per_product"] = nprod
                    roof["f32_equivalent_tflops"] = round(ach / nprod, 2)
        elif dom == "joiner":
            ach = f_join * nprof / cnt / per_launch_s / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2),
                    "peak": peak_mfma, "unit": "TFLOP/s", "frac": round(ach / peak_mfma, 4),
                    "traffic": None}
        else:
            # search step / decoder: one block per stream per frame, latency-bound
            roof = {"kernel": dom, "bound": "latency", "achieved": None, "peak": None,
                    "unit": None, "frac": None, "traffic": None}
        roof["avg_launch_ms"] = round(per_launch_s * 1e3, 4)
        roof["launches_per_step"] = cnt // nprof
        roof["timing"] = (f"HIP events around every launch of the class on its stream, over "
                          f"{nprof} extra profiled steps after the timed region (profile mode "
                          f"times each kernel alone; the timed steps above run the batch "
                          f"pipeline, where kernels of two batches overlap)")
        tr = pmc_traffic(dom, args)
        if tr is not None:
            roof["traffic"] = tr["bytes_per_launch"]
            roof["traffic_source"] = tr["source"]

    # fbank GB/s against HBM -- algorithmic bytes = the f32 samples read + the
    # f32 [T][80] features written, per step, over the class's HIP-event time
    fb_roof = None
    if "fbank" in classes:
        fb_bytes = sum(4 * n + 320 * ((n + 80) // 160) for n in lens)
        fb_s = classes["fbank"][1] / nprof * 1e-3
        fb_roof = {"bound": "hbm", "bytes_per_step": fb_bytes,
                   "ms_per_step": round(fb_s * 1e3, 4),
                   "achieved": round(fb_bytes / fb_s / 1e9, 1), "unit": "GB/s",
                   "peak": HBM_PEAK_GBS, "frac": round(fb_bytes / fb_s / 1e9 / HBM_PEAK_GBS, 4)}
    # the headline decode's tokens against the oracle's decode of the same hour (rank 0's
    # hour is the golden's; the other ranks decode seed + rank)
    ocheck = None
    if rec is not None and rank == 0 and not args.shard_plan:
        golden = hour_golden(args, beam, hotwords, chunks)
        if golden is not None:
            ocheck = oracle_agreement(golden[0], golden[1], [[r.token_ids.tolist() for r in res]],
                                      golden[2])
            ocheck["note"] = ("the headline precision's tokens vs the oracle (fp32); bf16 is "
                              "BASELINE config 2's arithmetic, not a token-exact mode -- the "
                              "token-exact figure is parity_mode")
    # the same K steps from HOST audio: pinned host memory, each batch's samples uploaded on the
    # engine's copy stream under the previous batch's work (zasr_decode_host_batches) -- the
    # reference's unit of work starts from the host waveform (core/asr_engine.py:2068)
    host_line = None
    if rec is not None and not args.no_pipeline and not args.shard_plan and lens:
        h_wav = torch.from_numpy(np.concatenate(chunks)).pin_memory()
        n = len(lens)

        def hsteps(k):
            return rec.decode_host_batches(h_wav.data_ptr(), offs * k, lens * k, [n] * k,
                                           beam=beam, stream=stream)
        hsteps(1)
        sync()
        if dist:
            dist.barrier()
        sync()
        t1 = time.perf_counter()
        hres = hsteps(args.steps)
        sync()
        el_h = time.perf_counter() - t1
        if dist:
            from zasr.shard import max_over_ranks
            el_h = max_over_ranks(el_h, device=dev)
        host_line = {"value": round(args.audio_sec * world * args.steps / el_h, 2),
                     "unit": "audio-sec/sec", "ms_per_step": round(1000 * el_h / args.steps, 3),
                     "steps": args.steps, "pinned_host_audio_bytes": int(h_wav.numel() * 4),
                     "tokens_equal_resident": all(a.token_ids.tolist() == b.token_ids.tolist()
                                                  for a, b in zip(hres[-n:], res[-n:])),
                     "note": "same workload with the waveforms in pinned host memory: each "
                             "batch's upload (PCIe) inside the timed region, on the engine's "
                             "copy stream under the previous batch's work"}
        del h_wav
    parity = None
    if (rec is not None and world == 1 and args.parity_precision != "none"
            and args.parity_precision != args.precision):
        parity = run_parity_child()
    # configs 3, 4 and 5 in the token-exact mode, each in its own child process, beside the
    # default config-2 line (bounded: a few steps each)
    subs = None
    if (rec is not None and world == 1 and not args.no_sub_lines and beam == 1 and
            args.model == "zipformer-68m" and args.audio_sec == 3600.0 and not args.shard_plan
            and args.parity_precision not in ("none",)):
        k_sub = str(max(1, min(args.steps, 5)))
        subs = {}
        try:
            subs["config3_f16x3"] = sub_line(run_sub_bench(
                ["--method", "modified_beam_search", "--beam", "8", "--hotwords-file", "default",
                 "--precision", args.parity_precision, "--parity-precision", "none",
                 "--no-cpu-baseline", "--no-sub-lines", "--steps", k_sub, "--warmup", "1"]))
        except Exception as e:  # reported, never fatal to the headline line
            subs["config3_f16x3"] = {"error": str(e)[:400]}
        try:
            subs["config4_rover_f16x3"] = sub_line(run_sub_bench(
                ["--stage", "rover", "--beam", "8", "--hotwords-file", "default",
                 "--precision", args.parity_precision, "--no-cpu-baseline", "--steps", k_sub,
                 "--warmup", "1"]))
        except Exception as e:
            subs["config4_rover_f16x3"] = {"error": str(e)[:400]}
        try:
            subs["config5_pipe_f16x3"] = sub_line(run_sub_bench(
                ["--stage", "pipe", "--precision", args.parity_precision, "--no-cpu-baseline",
                 "--steps", k_sub, "--warmup", "1"]))
        except Exception as e:
            subs["config5_pipe_f16x3"] = {"error": str(e)[:400]}

    if rank == 0:
        hw_tag = (f" + hotwords ({len(hotwords[0])} phrases of {os.path.basename(hw_path)})"
                  if hotwords else "")
        line = {
            "metric": "audio-sec/sec (xRT) Zipformer-68M offline decode",
            "value": round(value, 2), "unit": "audio-sec/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000 * el / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if args.shard_plan else "weak", "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (seeded 16 kHz speech-like audio, random-init Zipformer weights)",
            "config": {"workload": f"{args.model} {args.method}"
                                   f"{'' if beam == 1 else ' beam %d' % beam}{hw_tag}"
                                   ", batched planner chunks, 1 h per GPU",
                       "model": args.model, "weights": args.weights,
                       "emitting_frame_fraction": round(emitted / max(1, tprime), 4),
                       "chunks_per_gpu": len(chunks),
                       "chunk_sec_min_max": [round(min(lens) / SR, 2), round(max(lens) / SR, 2)],
                       "audio_sec_per_gpu": args.audio_sec,
                       "decoded_sec_per_gpu_incl_overlap": round(sum(lens) / SR, 1),
                       "parallelism": (f"dp{world} (one hour for the job: each rank decodes its "
                                       f"LPT share of the chunk plan, results gathered to every "
                                       f"rank in chunk order by a host object gather; strong "
                                       f"scaling)" if args.shard_plan else
                                       f"dp{world} (each rank its own hour, seed + rank; weak "
                                       f"scaling, no collective on the data path)"),
                       "shard_chunks_this_rank": len(chunks) if args.shard_plan else None,
                       "proxy_ranks": args.proxy_ranks or None,
                       "batch_pipeline": not args.no_pipeline,
                       "single_batch_latency_ms": (round(batch_latency_ms, 3)
                                                   if batch_latency_ms is not None else None),
                       "rtf": round(1.0 / (value / world), 8),
                       "tokens_emitted_per_gpu": emitted, "encoder_frames_per_gpu": tprime},
            "roofline": roof,
            "roofline_e2e": e2e,
            "kernel_classes_ms_per_step": {k: round(v[1] / nprof, 3) for k, v in classes.items()},
            "fbank_roofline": fb_roof,
            "cpu_baseline": cpu,
            "oracle_check": ocheck,
            "parity_mode": parity,
            "host_audio": host_line,
            "token_exact_lines": subs,
        }
        if args.cpu_dry_run:
            line["dry_run"] = True
        if shapes is not None:
            line["gemm_shapes"] = shapes
        print(json.dumps(line))
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump(line, f, indent=1)
    if rec is not None:
        rec.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
