"""Host models of the GEMM kernels' workgroup -> tile maps (csrc/gemm.hip), checked exhaustively on
the CPU: every launch must visit each (tile, K-slice) exactly once whatever the tile count, slice
count or grid, or a tile is silently lost / computed twice. The formulas below are the device code's,
line for line:

- gemm_nt_kernel: bijective XCD remap of blockIdx.x, then GROUP_M panel order (tile-major);
- gemm_nt_kernel with split-K and ctl bit kCtlSplitXcd: the same remap over (split, tile) in dispatch
  order, split-major, so an XCD's workgroups share one K-range (round 5);
- gemm_persist_kernel: workgroup b walks virtual ids b, b + G, ... through tile_coords.
"""
import itertools

import pytest

G_GROUP_M = 8


def xcd_remap(v, n):
    """the bijective XCD remap of csrc/gemm.hip: virtual id v of n -> contiguous range per XCD"""
    xcd, q, rr = v & 7, n >> 3, n & 7
    return (xcd * (q + 1) if xcd < rr else rr * (q + 1) + (xcd - rr) * q) + (v >> 3)


def group_m(wg, tiles_m, tiles_n):
    group = G_GROUP_M * tiles_n
    first_m = (wg // group) * G_GROUP_M
    gm = min(tiles_m - first_m, G_GROUP_M)
    return first_m + (wg % group) % gm, (wg % group) // gm


def nt_tiles(tiles_m, tiles_n, splits, split_xcd):
    nwg = tiles_m * tiles_n
    seen = []
    for y in range(splits):
        for bid in range(nwg):
            if split_xcd and splits > 1:
                L, nall = bid + nwg * y, nwg * splits
                v = xcd_remap(L, nall)
                split, wg = v // nwg, v % nwg
            else:
                split, wg = y, xcd_remap(bid, nwg)
            tm, tn = group_m(wg, tiles_m, tiles_n)
            assert 0 <= tm < tiles_m and 0 <= tn < tiles_n and 0 <= split < splits
            seen.append((split, tm, tn))
    return seen


SHAPES = [(1, 1), (1, 4), (4, 4), (12, 4), (16, 4), (7, 7), (25, 7), (3, 5), (384, 16), (57, 120)]


@pytest.mark.parametrize("tiles_m,tiles_n", SHAPES)
@pytest.mark.parametrize("splits", [1, 2, 3, 4, 16])
@pytest.mark.parametrize("split_xcd", [False, True])
def test_nt_kernel_visits_every_tile_and_slice_once(tiles_m, tiles_n, splits, split_xcd):
    seen = nt_tiles(tiles_m, tiles_n, splits, split_xcd)
    want = set(itertools.product(range(splits), range(tiles_m), range(tiles_n)))
    assert len(seen) == len(want) and set(seen) == want


def test_split_major_remap_keeps_an_xcds_workgroups_on_one_k_range():
    """The point of the split-major remap: at the FFN weight-gradient shape (64 tiles x 4 slices,
    one round of 256 workgroups) the 32 workgroups of each XCD (dispatch id mod 8) share one slice,
    and form an 8 x 4 tile block."""
    tiles_m, tiles_n, splits = 16, 4, 4
    nwg = tiles_m * tiles_n
    by_xcd = {}
    for y in range(splits):
        for bid in range(nwg):
            L = bid + nwg * y
            v = xcd_remap(L, nwg * splits)
            split, wg = v // nwg, v % nwg
            by_xcd.setdefault(L & 7, []).append((split,) + group_m(wg, tiles_m, tiles_n))
    for xcd, items in by_xcd.items():
        assert len(items) == 32
        assert len({s for s, _, _ in items}) == 1
        assert len({tm for _, tm, _ in items}) == 8 and len({tn for _, _, tn in items}) == 4


def persist_tiles(tiles_m, tiles_n, grid):
    nwg = tiles_m * tiles_n
    seen = []
    for b in range(grid):
        for v in range(b, nwg, grid):
            tm, tn = group_m(xcd_remap(v, nwg), tiles_m, tiles_n)
            seen.append((tm, tn))
    return seen


@pytest.mark.parametrize("tiles_m,tiles_n", [(384, 16), (384, 12), (384, 4), (57, 9), (2, 300)])
@pytest.mark.parametrize("grid", [256, 248, 64])
def test_persistent_walk_visits_every_tile_once(tiles_m, tiles_n, grid):
    seen = persist_tiles(tiles_m, tiles_n, grid)
    assert sorted(seen) == sorted(itertools.product(range(tiles_m), range(tiles_n)))
