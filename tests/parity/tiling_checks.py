"""Parity with ``heat/core/tests/test_tiling.py``: SplitTiles (tile grid = the chunking rule in every
dimension, tile owners, local get/set and errors) and SquareDiagTiles (row/column boundaries,
tiles per process, last diagonal process, tile access, local/global tile coordinates) including the
reference's fixed values at 3 ranks."""
import numpy as np
import torch

import heat_amd as ht

from ._util import raises


def test_raises():
    t = torch.arange(20 * 21, dtype=torch.float64).reshape(20, 21)
    tiles = ht.tiling.SplitTiles(ht.array(t, split=1))
    raises(TypeError, tiles.__getitem__, "p")
    raises(TypeError, tiles.__setitem__, 0, "p")
    raises(TypeError, tiles.__setitem__, "p", "p")


def test_misc_coverage():
    t = torch.arange(5 * 6 * 7, dtype=torch.float64).reshape(5, 6, 7)
    a = ht.array(t, split=None)
    tiles = ht.tiling.SplitTiles(a)
    assert torch.all(tiles.tile_locations == a.comm.rank)
    a = ht.resplit(a, 0)
    tiles = ht.tiling.SplitTiles(a)
    p, me = a.comm.size, a.comm.rank
    # tile grid: every dimension chunked like the split axis
    for d, n in enumerate((5, 6, 7)):
        dims = tiles.tile_dimensions[d].tolist()
        assert sum(dims) == n and dims == [n // p + (1 if r < n % p else 0) for r in range(p)]
    assert (tiles.tile_locations.select(0, 0) == 0).all() and (tiles.tile_locations.select(0, p - 1) == p - 1).all()
    if p == 3:
        assert torch.equal(tiles.tile_dimensions.float(), torch.tensor([[2.0, 2.0, 1.0], [2.0, 2.0, 2.0],
                                                                        [3.0, 2.0, 2.0]]))
        if me == 2:
            assert torch.equal(tiles[2], t[4:5])
    last = max(i for i in range(p) if tiles.tile_dimensions[0, i] > 0)
    lo = sum(tiles.tile_dimensions[0, :last].tolist())
    tiles[last] = 1000
    sl = tiles[last]
    if me == last:
        assert sl.shape == (tiles.tile_dimensions[0, last].item(), 6, 7) and torch.all(sl == 1000)
    elif p > 1:
        assert sl is None
    full = a.numpy()
    assert (full[lo:] == 1000).all() and (full[:lo] == t.numpy()[:lo]).all()
    # tiles of a tile range along several dimensions
    b = ht.array(t, split=2)
    tb = ht.tiling.SplitTiles(b)
    piece = tb[0, :, 0]
    if me == 0:
        d = tb.tile_dimensions
        assert piece.shape == (d[0, 0].item(), 6, d[2, 0].item())
    assert tb.get_tile_size((0, 0, 0)) == tuple(int(tb.tile_dimensions[i, 0]) for i in range(3))


def _sq_invariants(arr, tiles, tpp):
    m, n = arr.gshape
    rows, cols = tiles.row_indices, tiles.col_indices
    assert rows == sorted(rows) and cols == sorted(cols) and rows[0] == 0 and cols[0] == 0
    assert tiles.tile_rows == len(rows) and tiles.tile_columns == len(cols)
    assert torch.equal(tiles.lshape_map, arr.create_lshape_map())
    assert ht.equal(tiles.arr, arr)
    # tiles cover the array: reassemble it from the tile getter
    rec = np.zeros((m, n))
    full = arr.numpy()
    for i in range(tiles.tile_rows):
        for j in range(tiles.tile_columns):
            r0, r1, c0, c1 = tiles.get_start_stop((i, j))
            assert 0 <= r0 <= r1 <= m and 0 <= c0 <= c1 <= n
            rec[r0:r1, c0:c1] += 1
            loc = tiles[i, j]
            if loc is not None and loc.numel():
                # the local piece holds exactly the global values of that tile region
                assert np.isin(loc.cpu().numpy(), full[r0:r1, c0:c1]).all()
    assert (rec == 1).all()


def test_init_raises():
    raises(TypeError, ht.core.tiling.SquareDiagTiles, "sdkd", tiles_per_proc=1)
    raises(TypeError, ht.core.tiling.SquareDiagTiles, ht.arange(2), tiles_per_proc="sdf")
    raises(ValueError, ht.core.tiling.SquareDiagTiles, ht.arange(2), tiles_per_proc=0)
    raises(ValueError, ht.core.tiling.SquareDiagTiles, ht.arange(2), tiles_per_proc=1)


def test_properties():
    p = ht.MPI_WORLD.size
    for shape in ((47, 47), (38, 128), (128, 38)):
        for split in (0, 1):
            arr = ht.array(np.random.default_rng(1).standard_normal(shape), split=split)
            for tpp in (1, 2):
                t = ht.tiling.SquareDiagTiles(arr, tiles_per_proc=tpp)
                _sq_invariants(arr, t, tpp)
                if shape == (47, 47):
                    assert t.last_diagonal_process == p - 1
                    assert t.tile_columns == p * tpp and t.tile_rows == p * tpp
                if p == 3 and shape == (47, 47):
                    exp = [0, 16, 32] if tpp == 1 else [0, 8, 16, 24, 32, 40]
                    assert t.col_indices == exp and t.row_indices == exp
                    if split == 0:
                        assert t.tile_columns_per_process == [3 * tpp] * 3
                        assert t.tile_rows_per_process == [tpp] * 3
                    else:
                        assert t.tile_columns_per_process == [tpp] * 3
                        assert t.tile_rows_per_process == [3 * tpp] * 3
                if p == 3 and shape == (38, 128) and split == 0:
                    exp = [0, 13, 26] if tpp == 1 else [0, 7, 13, 20, 26, 32]
                    assert t.col_indices == exp and t.row_indices == exp


def test_local_set_get():
    arr = ht.zeros((23, 23), split=0)
    t = ht.tiling.SquareDiagTiles(arr, tiles_per_proc=2)
    me = arr.comm.rank
    t.local_set((0, 0), 5.0)
    g = t.local_to_global((0, 0), me)
    r0, r1, c0, c1 = t.get_start_stop(g)
    full = arr.numpy()
    counts = arr.create_lshape_map()[:, 0].tolist()
    off = 0
    for q in range(arr.comm.size):
        if counts[q]:
            gq = t.local_to_global((0, 0), q)
            a0, a1, b0, b1 = t.get_start_stop(gq)
            assert (full[a0:a1, b0:b1] == 5).all()
    loc = t.local_get(g)
    assert loc is not None and torch.all(loc == 5)
    assert float(arr.sum().item()) == 5.0 * sum(
        (lambda s: (s[1] - s[0]) * (s[3] - s[2]))(t.get_start_stop(t.local_to_global((0, 0), q)))
        for q in range(arr.comm.size) if counts[q])
    other = ht.tiling.SquareDiagTiles(ht.zeros((23, 30), split=0), tiles_per_proc=1)
    t.match_tiles(other)
    assert t.row_indices == [r for r in other.row_indices if r < 23]
    raises(TypeError, t.match_tiles, "x")
