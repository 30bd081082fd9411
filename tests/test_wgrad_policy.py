"""Weight-gradient routing (apex.ops.fused): which shapes go to the transposed-read MFMA kernel
(_wgrad_tt_splits) and how the library split-K slices (_wgrad_splits) are chosen. Pure host logic."""
import torch

from apex.ops import fused


def test_tt_auto_takes_the_ffn_shapes_only(monkeypatch):
    monkeypatch.setattr(fused, "_WGRAD_TT", "auto")
    M = 98304
    assert fused._wgrad_tt_splits(M, 4096, 1024) == 4  # FFN1: 64 tiles -> one wave of 256 workgroups
    assert fused._wgrad_tt_splits(M, 1024, 4096) == 4  # FFN2
    assert fused._wgrad_tt_splits(M, 3072, 1024) == 0  # QKV (48 tiles): library
    assert fused._wgrad_tt_splits(M, 1024, 1024) == 16  # attention out (16 tiles): measured, 16 slices
    assert fused._wgrad_tt_splits(32768, 1024, 1024) == 0  # ... below its measured token count: library
    assert fused._wgrad_tt_splits(16384, 1600, 1600) == 4  # GPT-2 1.5B attention out: measured
    assert fused._wgrad_tt_splits(8192, 4096, 1024) == 0  # too few tokens
    assert fused._wgrad_tt_splits(M, 1600, 4800) == 0  # partial tiles, unmeasured: library
    assert fused._wgrad_tt_splits(M, 2560, 7680) == 0  # 300 tiles: unmeasured, library


def test_tt_table_from_env():
    assert fused._parse_tt_table("none") == {}
    assert fused._parse_tt_table("1024x1024:65536:16, 1600x6400:16384:4") == {(1024, 1024): (65536, 16),
                                                                               (1600, 6400): (16384, 4)}
    import pytest

    with pytest.raises(ValueError, match="APEX_WGRAD_TT_TABLE"):
        fused._parse_tt_table("1024x1024:16")


def test_tt_overrides(monkeypatch):
    monkeypatch.setattr(fused, "_WGRAD_TT", "0")
    assert fused._wgrad_tt_splits(98304, 4096, 1024) == 0
    monkeypatch.setattr(fused, "_WGRAD_TT", "8")
    assert fused._wgrad_tt_splits(98304, 3072, 1024) == 8
    # slices are whole 64-row K-tiles, any count up to the K-tile count (uneven slices allowed)
    assert fused._wgrad_tt_splits(98304 + 64, 3072, 1024) == 8
    assert fused._wgrad_tt_splits(98304 + 32, 3072, 1024) == 0  # rows not a whole number of K-tiles
    assert fused._wgrad_tt_splits(448, 3072, 1024) == 0  # 7 K-tiles: fewer than 8 slices
    assert fused._wgrad_tt_splits(16384, 4800, 1600) == 8  # partial tiles: the forced count applies
    monkeypatch.setattr(fused, "_WGRAD_TT", "auto")
    assert fused._wgrad_tt_splits(16384, 4800, 1600) == 0  # GPT-2 QKV: the library wins it
    assert fused._wgrad_tt_splits(16384, 6400, 1600) == 0  # GPT-2 FFN: faster alone, slower in the model
    monkeypatch.setattr(fused, "_WGRAD_TT_MEASURED", {(6400, 1600): (16384, 4)})
    assert fused._wgrad_tt_splits(16384, 6400, 1600) == 4  # a measured entry routes its shape
    assert fused._wgrad_tt_splits(8192, 6400, 1600) == 0  # ... from its token count up


def test_library_split_k_fills_the_chip(monkeypatch):
    monkeypatch.setattr(fused, "_WGRAD_SPLITK", "auto")
    M = 98304
    for n, k in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        s = fused._wgrad_splits(M, n, k)
        tiles = ((n + 255) // 256) * ((k + 255) // 256)
        assert M % s == 0 and s * tiles <= 256 and (s == 16 or 2 * s * tiles > 256)
    assert fused._wgrad_splits(4096, 1024, 1024) == 1


def test_vocab_sized_weight_gradients_take_the_kernel(monkeypatch):
    """An MLM decoder / LM head weight (vocabulary rows) goes to the transposed-read kernel in one
    slice; APEX_WGRAD_TT_VOCAB=0 leaves it on the library."""
    monkeypatch.setattr(fused, "_WGRAD_TT", "auto")
    monkeypatch.setattr(fused, "_WGRAD_TT_VOCAB", True)
    assert fused._wgrad_tt_splits(14592, 30528, 1024) == 1  # BERT-Large MLM decoder, b768
    assert fused._wgrad_tt_splits(16384, 50304, 1600) == 1  # GPT-2 LM head
    assert fused._wgrad_tt_splits(14590, 30528, 1024) == 0  # tokens not a multiple of 64
    monkeypatch.setattr(fused, "_WGRAD_TT_VOCAB", False)
    assert fused._wgrad_tt_splits(14592, 30528, 1024) == 0


def test_vocab_routing_is_keyed_on_measured_weight_shapes(monkeypatch):
    """Plain forward / input-gradient products go to the MFMA kernel only for the measured
    vocabulary projections (weight shape), never for an unmeasured wide layer (16384-wide FFN)."""
    from apex.ops import gemm as G

    assert G._vocab_sized(torch.empty(30528, 1024))  # BERT-Large MLM decoder
    assert not G._vocab_sized(torch.empty(16384, 4096))  # FFN1 of a hidden-4096 model
    assert not G._vocab_sized(torch.empty(4096, 16384))  # its FFN2
    assert not G._vocab_sized(torch.empty(50304, 1600))  # GPT-2 LM head: measured neutral
    assert G._parse_shapes("none") == set()
    assert G._parse_shapes("50304x1600, 30528x1024") == {(50304, 1600), (30528, 1024)}
