"""N > 1 path on CPU: world-size-2 (and 8) gloo process groups (one process per GPU on the box).

Covers zasr.shard (LPT split, ordered gather, max-over-ranks timing), the drop-in
decode_chunks sharding with a fake recognizer handle (no GPU needed), and the strong-scaling
forms of BASELINE configs 4 and 5: the sharded ROVER pass (zasr.rover.rover_device_many with
`mine`) and the row-sharded ViBERT session under the config-5 restorer must give every rank
exactly the single-process result."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "sherpa-vietnamese-asr_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeResult:
    def __init__(self, n):
        k = n % 5
        self.token_ids = np.arange(3, 3 + k, dtype=np.int32)
        self.frames = np.arange(k, dtype=np.int32) * 2
        self.log_probs = np.full(k, -0.1, np.float64)
        self.T = max(1, n // 640)
        self.stats = np.tile(np.array([[0.5, 20.0, 0.9, 0.05]], np.float32), (k, 1))


class _FakeHandle:
    def __init__(self):
        self.seen = []

    def decode(self, chunks, beam=8):
        self.seen.extend(len(c) for c in chunks)
        return [_FakeResult(len(c)) for c in chunks]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zasr.shard import decode_sharded, lpt_partition, max_over_ranks
    from zasr.asr_engine import decode_chunks
    lens = [16000 * s + 37 * i for i, s in enumerate((30, 22, 33, 5, 28, 31, 20))]
    chunks = [np.full(n, 0.01 * i, np.float32) for i, n in enumerate(lens)]
    # ordered gather of an identity decode
    got = decode_sharded(lambda cs: [len(c) for c in cs], chunks)
    assert got == lens, got
    # this rank decoded exactly its LPT share
    share = lpt_partition(lens, world)[rank]
    h = _FakeHandle()
    rec = {"handle": h, "max_active_paths": 8, "id2token": {i: "▁w%d" % i for i in range(64)},
           "vocab_size": 64}
    words = decode_chunks(rec, chunks, [float(i) for i in range(len(chunks))])
    assert sorted(h.seen) == sorted(lens[i] for i in share), (h.seen, share)
    assert len(words) == len(chunks)
    # time offsets stay attached to their chunks
    for i, w in enumerate(words):
        for x in w:
            assert x["start"] >= i - 1e-9
    t = max_over_ranks(1.0 + rank)
    assert t == float(world), t
    with open(os.path.join(out_dir, "rank%d.ok" % rank), "w") as f:
        f.write("%d words\n" % sum(len(w) for w in words))
    dist.barrier()
    dist.destroy_process_group()


def test_lpt_partition_balances_and_covers():
    sys.path.insert(0, PKG)
    from zasr.shard import lpt_partition
    lens = [9, 8, 7, 6, 5, 4, 3, 2, 1]
    parts = lpt_partition(lens, 3)
    assert sorted(i for p in parts for i in p) == list(range(9))
    loads = [sum(lens[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= 2  # LPT: 16, 15, 14
    assert lpt_partition(lens, 1) == [list(range(9))]
    assert lpt_partition([], 2) == [[], []]
    with pytest.raises(ValueError):
        lpt_partition(lens, 0)


def test_world2_gloo_sharded_decode(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / ("rank%d.ok" % r)).exists()


class _FakeDeviceHandle:
    """decode_device / decode_device_batches over (offset, length) pairs: a result that
    depends only on the chunk (its offset and length) and the model seed."""

    def __init__(self, seed):
        self.seed = seed
        self.seen = []

    def _one(self, off, n):
        rng = np.random.default_rng([self.seed, off, n])
        k = int(rng.integers(2, 9))
        r = _FakeResult(n)
        r.token_ids = rng.integers(3, 60, k).astype(np.int32)
        r.frames = np.sort(rng.choice(np.arange(max(k, n // 640)), k, replace=False)).astype(np.int32)
        r.log_probs = -rng.random(k)
        r.T = max(k, n // 640)
        r.stats = np.tile(np.array([[0.5, 20.0, 0.9, 0.05]], np.float32), (k, 1))
        return r

    def decode_device(self, d_wav, offsets, lengths, beam=8, stream=0):
        self.seen.extend(zip(offsets, lengths))
        return [self._one(o, n) for o, n in zip(offsets, lengths)]

    def decode_device_batches(self, d_wav, offsets, lengths, sizes, beam=8, stream=0):
        return self.decode_device(d_wav, offsets, lengths, beam)


class _FakeVibert:
    """ONNX-session surface: per-row outputs computed from that row alone."""

    def run(self, names, feeds):
        ids = feeds["input_ids"].astype(np.float64)
        B, L = ids.shape
        logits = np.stack([np.sin(ids * (c + 1) * 0.37) for c in range(15)], -1).astype(np.float32)
        detect = np.stack([np.cos(ids * 0.11), np.sin(ids * 0.13)], -1).astype(np.float32)
        return [logits, detect]


def _rover_pipe_reference():
    """The single-process results the sharded ranks must reproduce."""
    sys.path.insert(0, PKG)
    from zasr.pipeline import make_punctuator, transcript_for_punctuation
    from zasr.rover import rover_device_many
    lens = [16000 * s + 131 * i for i, s in enumerate((30, 22, 33, 5, 28, 31, 20, 27, 29))]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    recd = {"id2token": {i: ("▁w%d" % i if i % 3 else "p%d" % i) for i in range(64)},
            "vocab_size": 64}
    out = rover_device_many(_FakeDeviceHandle(1), _FakeDeviceHandle(2), recd, recd, 0, offs,
                            lens, 2, 8, ["w5 w7"])
    words = out[-1][0]
    text, hints = transcript_for_punctuation(words)
    punct = make_punctuator(_FakeVibert(), 64, mini_batch=0)
    return lens, offs, recd, words, punct.restore(text, pause_hints=hints)


def _shard_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    sys.path.insert(0, PKG)
    import json
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zasr.pipeline import make_punctuator, transcript_for_punctuation
    from zasr.rover import rover_device_many
    from zasr.shard import RowShardedSession, gather_chunks, lpt_partition
    lens, offs, recd, ref_words, ref_text = _rover_pipe_reference()
    mine = lpt_partition(lens, world)[rank]
    ha, hb = _FakeDeviceHandle(1), _FakeDeviceHandle(2)
    out = rover_device_many(ha, hb, recd, recd, 0, offs, lens, 2, 8, ["w5 w7"], mine=mine)
    assert sorted(n for _, n in ha.seen) == sorted([lens[i] for i in mine] * 2)
    words = out[-1][0]
    assert json.dumps(words, sort_keys=True) == json.dumps(ref_words, sort_keys=True)
    # config 5: every rank runs the restorer on the gathered transcript, ViBERT rows split
    text, hints = transcript_for_punctuation(words)
    punct = make_punctuator(RowShardedSession(_FakeVibert()), 64, mini_batch=0)
    assert punct.restore(text, pause_hints=hints) == ref_text
    # ordered gather with an empty share on some ranks
    got = gather_chunks([(i, i * 10) for i in range(rank, 3, world)], 3)
    assert got == [0, 10, 20]
    with open(os.path.join(out_dir, "rank%d.ok" % rank), "w") as f:
        f.write("%d words\n" % len(words))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_rover_and_punctuation_equal_single_process(tmp_path, world):
    """--shard-plan for configs 4 and 5 (bench.py --stage rover / pipe): chunks decoded and
    voted per rank, voted chunks gathered in chunk order, merge on every rank; the restorer's
    ViBERT runs split by rows over the ranks -- words and punctuated text identical to one
    process, at 2 and 8 ranks (more ranks than some shares have chunks)."""
    import torch.multiprocessing as mp
    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / ("rank%d.ok" % r)).exists()
