"""bench.py --gpus N: the launcher path the driver uses, on CPU.

`python bench.py --gpus 2 ...` without RANK starts torch.distributed.run with 2 ranks as a
child process; each rank plans its own synthetic audio, the timed region is bracketed by
barriers and the time is max-reduced over ranks (gloo here, RCCL on the box).  --cpu-dry-run
replaces the GPU decode with a CPU stand-in so the whole path runs without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--cpu-dry-run",
                        "--steps", "2", "--warmup", "1", "--audio-sec", "40",
                        "--no-cpu-baseline", *extra],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    line = _run("--gpus", "2")
    assert line["n_gpus"] == 2
    assert line["scaling"] == "weak"
    assert line["dry_run"] is True
    assert line["config"]["parallelism"].startswith("dp2")


def test_bench_single_rank_default():
    line = _run()
    assert line["n_gpus"] == 1
    assert line["config"]["chunks_per_gpu"] >= 1
    assert 20.0 <= line["config"]["chunk_sec_min_max"][1] <= 36.0


def test_bench_shard_plan_two_ranks_strong_scaling():
    """--shard-plan: both ranks plan the same audio, decode their LPT shares, gather every
    chunk's result in chunk order (gloo object gather here) inside the timed region; the line
    reports strong scaling and the job's audio once (not x ranks)."""
    one = _run("--shard-plan")
    two = _run("--gpus", "2", "--shard-plan")
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert "LPT share" in two["config"]["parallelism"]
    # the gathered hour: every chunk's result, the same token count as the single-rank run
    assert two["config"]["tokens_emitted_per_gpu"] == one["config"]["tokens_emitted_per_gpu"]
    assert two["config"]["shard_chunks_this_rank"] < one["config"]["shard_chunks_this_rank"]
    # value = audio of the job / time (x1, not x world)
    assert abs(two["value"] - 40.0 * two["steps"] / (two["ms_per_step"] * two["steps"] / 1e3)) \
        <= 0.02 * two["value"]


def test_bench_gpus8_shard_plan():
    """The 8-rank launch the driver runs at round end (SCALE), on CPU: 8 gloo ranks, the hour's
    chunks LPT-split 8 ways and gathered in chunk order."""
    one = _run("--shard-plan")
    eight = _run("--gpus", "8", "--shard-plan")
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
    assert eight["config"]["tokens_emitted_per_gpu"] == one["config"]["tokens_emitted_per_gpu"]


def test_bench_proxy_ranks_single_gpu():
    """--proxy-ranks 8 (DESIGN §9's single-GPU proxy): one process decodes the largest of the
    8 LPT shares of the hour; strong-scaling line, the job's audio over that share's time."""
    one = _run("--shard-plan")
    proxy = _run("--proxy-ranks", "8")
    assert proxy["n_gpus"] == 1 and proxy["scaling"] == "strong"
    assert proxy["config"]["proxy_ranks"] == 8
    assert 1 <= proxy["config"]["shard_chunks_this_rank"] < one["config"]["shard_chunks_this_rank"]
