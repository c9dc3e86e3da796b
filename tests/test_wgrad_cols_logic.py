"""Host logic of the column-split weight-gradient route (mlp._col_split): which layers take two
single-tile launches, and where the cut falls (tests/test_gpu_wgrad_cols.py runs them)."""
from nerf_amd import mlp


def _segs(*ks):
    return [(None, k, 1) for k in ks]


def test_col_split_cuts():
    assert mlp._col_split(_segs(256, 96), 256) == 1          # mip's skip layer
    assert mlp._col_split(_segs(256, 63), 257) == 1          # padded encoding, 257 output rows
    assert mlp._col_split(_segs(128, 128, 60), 256) == 2
    assert mlp._col_split(_segs(192, 96, 27), 200) == 1      # 192 | 96 + 27 -> 128


def test_col_split_declines():
    assert mlp._col_split(_segs(256), 256) is None            # one tile already
    assert mlp._col_split(_segs(192, 60), 256) is None        # 256 padded columns: one tile
    assert mlp._col_split(_segs(256, 96), 128) is None        # few output rows: the 128-tile kernel
    assert mlp._col_split(_segs(256, 96), 260) is None        # 257 rows padded to 260: no single tile
    assert mlp._col_split(_segs(256, 256, 32), 256) is None   # the rest exceeds one tile
    assert mlp._col_split(_segs(300, 32), 256) is None        # first segment alone exceeds one tile
    saved = mlp.WGRAD_COLSPLIT
    mlp.WGRAD_COLSPLIT = False
    try:
        assert mlp._col_split(_segs(256, 96), 256) is None
    finally:
        mlp.WGRAD_COLSPLIT = saved
