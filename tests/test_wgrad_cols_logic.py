"""Host logic of the tile-split weight-gradient route (mlp._tile_split): which layers take
single-tile launches, their row blocks and column groups (tests/test_gpu_wgrad_cols.py runs them)."""
from nerf_amd import mlp


def _segs(*ks, rd=1):
    return [(None, k, rd) for k in ks]


def test_tile_split_column_groups():
    assert mlp._tile_split(_segs(256, 96), 256) == ([(0, 256)], [[(0, 0, 256)], [(1, 0, 96)]])  # mip skip layer
    assert mlp._tile_split(_segs(256, 60), 257) == ([(0, 257)], [[(0, 0, 256)], [(1, 0, 60)]])  # 257 rows
    assert mlp._tile_split(_segs(128, 128, 60), 256)[1] == [[(0, 0, 128), (1, 0, 128)], [(2, 0, 60)]]
    assert mlp._tile_split(_segs(192, 96, 24), 200)[1] == [[(0, 0, 192)], [(1, 0, 96), (2, 0, 24)]]
    # a segment wider than a tile: 256-column slices (GARF's Linear(1024, 256))
    assert mlp._tile_split(_segs(1024), 256)[1] == [[(0, c, c + 256)] for c in range(0, 1024, 256)]
    assert mlp._tile_split(_segs(128, 512), 256)[1] == [[(0, 0, 128)], [(1, 0, 256)], [(1, 256, 512)]]


def test_tile_split_row_blocks():
    # GARF's Linear(131, 512) (model_radiance.py): two row blocks, one 160-column group
    assert mlp._tile_split(_segs(128, 4), 512) == ([(0, 256), (256, 256)], [[(0, 0, 128), (1, 0, 4)]])
    assert mlp._tile_split(_segs(512), 512) == ([(0, 256), (256, 256)], [[(0, 0, 256)], [(0, 256, 512)]])


def test_tile_split_declines():
    assert mlp._tile_split(_segs(256), 256) is None            # one tile already
    assert mlp._tile_split(_segs(192, 60), 257) is None        # 256 padded columns, 257 rows: one tile
    assert mlp._tile_split(_segs(4), 1024) is None             # row blocks of a narrow input (Linear(3, 1024))
    assert mlp._tile_split(_segs(256, 96), 1024) is None       # row blocks with a 96-column group
    assert mlp._tile_split(_segs(256, 96), 128) is None        # 128 rows x 96 columns: no single tile
    assert mlp._tile_split(_segs(512, rd=64), 256) is None     # a wide per-ray segment is not sliced
    saved = mlp.WGRAD_TILESPLIT
    mlp.WGRAD_TILESPLIT = False
    try:
        assert mlp._tile_split(_segs(256, 96), 256) is None
    finally:
        mlp.WGRAD_TILESPLIT = saved
