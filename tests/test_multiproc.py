"""N > 1 path on CPU: world-size-2 gloo process group (one process per GPU on the box).

Covers zasr.shard (LPT split, ordered gather, max-over-ranks timing) and the drop-in
decode_chunks sharding with a fake recognizer handle (no GPU needed)."""
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
