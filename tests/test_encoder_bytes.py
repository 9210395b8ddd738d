"""Reconciling the restated architecture with the only reference-held facts about the
graphs: the byte sizes of the ONNX files (offline_pwa/model_manifest.json:21, 30, 39 (30M)
and :73, 82, 91 (68M); the numbers are copied here, the reference never travels).  DESIGN.md
§4c walks through the accounting; this test keeps it true.

  file bytes = 4 x restated parameters                     (f32 initializers)
             + 6 x CompactRelPositionalEncoding table       (traced constant, see below)
             + graph serialization                          (node protos, names, attributes)

* decoder / joiner: parameters are 5,163,008 / 4,104,000 B against 5,165,084 / 4,104,465 B:
  2,076 B and 465 B of graph for graphs of a handful of nodes.
* encoders: the restated parameters are 257,003,996 B (68M) and 88,473,676 B (30M).  Each of
  the 6 encoder stacks holds a CompactRelPositionalEncoding whose table is computed at
  construction for max_len 1000 -- (2*1000 - 1) x pos_dim 48 f32 = 383,808 B -- and is a plain
  tensor attribute (not a parameter), so the trace bakes it into the graph as a constant
  sliced at run time: 2,302,848 B per encoder, the same in both models.
* what remains, 1,750,848 B (68M, 16 layers) and 1,407,608 B (30M, 12 layers), is not a
  multiple of 4 per layer (not tensors) and fits 85,810 B per Zipformer2 layer + 377,888 B
  per encoder: for a traced layer of a few hundred nodes whose names and outputs are
  scope paths ("/encoder/encoders.3/encoder/layers.2/self_attn_weights/Reshape_3_output_0"),
  i.e. ~150-250 B per node.  The fit has two unknowns and two files, so it is a consistency
  statement, not a proof; a missing parameter tensor of >= 4 B per layer-channel would break
  the non-negativity and per-node plausibility bounds asserted here."""
import math

import pytest

from zasr.model import count_params, zipformer_m, zipformer_s

MANIFEST = {  # offline_pwa/model_manifest.json "bytes"
    "zipformer-68m": {"encoder": 261057692, "decoder": 5165084, "joiner": 4104465},
    "zipformer-30m": {"encoder": 92184132, "decoder": 5165084, "joiner": 4104465},
}
PE_MAX_LEN = 1000  # icefall CompactRelPositionalEncoding(max_len=1000)


def _enc_params(cfg):
    return sum(count_params(cfg, p) for p in ("encoder_embed.", "encoder.", "encoder_proj."))


def pe_bytes(cfg):
    from oracle.zipformer import compact_rel_pos_emb
    table = compact_rel_pos_emb(PE_MAX_LEN, cfg.pos_dim)
    return cfg.num_stacks * table.numel() * 4


@pytest.mark.parametrize("cfg_fn", [zipformer_m, zipformer_s])
def test_decoder_joiner_within_graph_overhead(cfg_fn):
    cfg = cfg_fn()
    m = MANIFEST[cfg.name]
    dec = 4 * (count_params(cfg, "decoder.") + count_params(cfg, "decoder_proj."))
    join = 4 * count_params(cfg, "joiner.")
    assert 0 < m["decoder"] - dec <= 4096 and 0 < m["joiner"] - join <= 4096
    assert (m["decoder"] - dec, m["joiner"] - join) == (2076, 465)


def test_encoder_bytes_decompose():
    rows = {}
    for cfg in (zipformer_m(), zipformer_s()):
        p = 4 * _enc_params(cfg)
        gap = MANIFEST[cfg.name]["encoder"] - p
        pe = pe_bytes(cfg)
        assert pe == 6 * 1999 * 48 * 4 == 2302848
        rest = gap - pe
        assert rest > 0, (cfg.name, gap, pe)
        rows[cfg.name] = (p, gap, rest, sum(cfg.num_layers))
    assert rows["zipformer-68m"][:2] == (257003996, 4053696)
    assert rows["zipformer-30m"][:2] == (88473676, 3710456)
    (r68, l68), (r30, l30) = (rows["zipformer-68m"][2:], rows["zipformer-30m"][2:])
    per_layer = (r68 - r30) / (l68 - l30)
    fixed = r68 - l68 * per_layer
    assert (per_layer, fixed) == (85810.0, 377888.0)
    # not tensor data (85,810 B is not a whole number of f32 values), and a few hundred
    # ~150-250 B node protos per layer
    assert per_layer % 4 != 0
    assert 40_000 <= per_layer <= 200_000 and 0 <= fixed <= 1_000_000


def test_pe_table_is_the_oracle_formula():
    """The table counted above is the one the oracle slices (relative offsets -(T-1)..T-1):
    the middle 2T-1 rows of the max_len table equal compact_rel_pos_emb(T)."""
    from oracle.zipformer import compact_rel_pos_emb
    full = compact_rel_pos_emb(PE_MAX_LEN, 48)
    T = 137
    mid = full.shape[0] // 2
    assert full.shape == (1999, 48)
    assert (full[mid - T + 1: mid + T] == compact_rel_pos_emb(T, 48)).all()
    assert math.isclose(float(full[mid, 0]), 1.0)
