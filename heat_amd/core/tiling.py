"""
Tile views of DNDarrays (reference ``heat/core/tiling.py``: ``SplitTiles`` 14, ``SquareDiagTiles``
331).

``SplitTiles`` divides EVERY dimension like the split axis would be divided (the chunking rule),
so tile (i, j, ...) of a split array lives on the rank owning block i of the split axis. It is the
tile grid behind resplit. ``SquareDiagTiles`` provides square diagonal tiles for tiled matrix
algorithms (tile bookkeeping with the reference's boundaries: ``tiles_per_proc`` tiles per rank
along the split axis, the other axis cut at the same indices).
"""
from __future__ import annotations

from typing import List, Tuple, Union

import torch

from .dndarray import DNDarray

__all__ = ["SplitTiles", "SquareDiagTiles"]


def _ends(n: int, p: int) -> List[int]:
    base, rem = divmod(n, p)
    out, s = [], 0
    for r in range(p):
        s += base + (1 if r < rem else 0)
        out.append(s)
    return out


class SplitTiles:
    """Tiles whose boundaries are the theoretical split boundaries in every dimension."""

    def __init__(self, arr: DNDarray) -> None:
        self.__DNDarray = arr
        p = arr.comm.size
        self.__lshape_map = arr.create_lshape_map()
        ends = [_ends(s, p) for s in arr.gshape]
        self.__tile_ends_g = torch.tensor(ends, dtype=torch.int32).reshape(arr.ndim, p)
        dims = torch.zeros_like(self.__tile_ends_g)
        dims[:, 0] = self.__tile_ends_g[:, 0]
        dims[:, 1:] = self.__tile_ends_g[:, 1:] - self.__tile_ends_g[:, :-1]
        self.__tile_dims = dims
        self.__tile_locations = self.set_tile_locations(arr.split, dims, arr)

    @staticmethod
    def set_tile_locations(split: int, tile_dims: torch.Tensor, arr: DNDarray) -> torch.Tensor:
        """Rank holding every tile: the tile index along the split axis (own rank if replicated)."""
        p = arr.comm.size
        shape = [p] * arr.ndim
        if split is None or not arr.comm.is_distributed():
            return torch.full(shape, arr.comm.rank, dtype=torch.int32)
        idx = torch.arange(p, dtype=torch.int32)
        view = [1] * arr.ndim
        view[split] = p
        return idx.reshape(view).expand(shape).clone()

    @property
    def arr(self) -> DNDarray:
        return self.__DNDarray

    @property
    def lshape_map(self) -> torch.Tensor:
        return self.__lshape_map

    @property
    def tile_locations(self) -> torch.Tensor:
        return self.__tile_locations

    @property
    def tile_ends_g(self) -> torch.Tensor:
        return self.__tile_ends_g

    @property
    def tile_dimensions(self) -> torch.Tensor:
        return self.__tile_dims

    def _tile_slices(self, key) -> Tuple[slice, ...]:
        """Global slices of the tile(s) addressed by ``key`` (ints or slices over the tile grid)."""
        arr = self.__DNDarray
        if not isinstance(key, tuple):
            key = (key,)
        key = list(key) + [slice(None)] * (arr.ndim - len(key))
        ends = self.__tile_ends_g
        out = []
        for d, k in enumerate(key):
            starts = [0] + ends[d, :-1].tolist()
            stops = ends[d].tolist()
            if isinstance(k, int):
                k = k + len(stops) if k < 0 else k
                out.append(slice(starts[k], stops[k]))
            elif isinstance(k, slice):
                idx = list(range(len(stops)))[k]
                if not idx:
                    out.append(slice(0, 0))
                else:
                    out.append(slice(starts[idx[0]], stops[idx[-1]]))
            else:
                raise TypeError("key must be int or slice, got {}".format(type(k)))
        return tuple(out)

    def __getitem__(self, key) -> torch.Tensor:
        """The process-local part of the addressed tile(s) (None if this rank holds none of it)."""
        arr = self.__DNDarray
        sl = list(self._tile_slices(key))
        if arr.split is None or not arr.comm.is_distributed():
            return arr.larray[tuple(sl)]
        s = arr.split
        counts, displs = arr.counts_displs()
        me = arr.comm.rank
        lo, hi = max(sl[s].start, displs[me]), min(sl[s].stop, displs[me] + counts[me])
        if hi <= lo:
            return None
        sl[s] = slice(lo - displs[me], hi - displs[me])
        return arr.larray[tuple(sl)]

    def get_tile_size(self, key) -> Tuple[int, ...]:
        return tuple(s.stop - s.start for s in self._tile_slices(key))

    def __setitem__(self, key, value):
        arr = self.__DNDarray
        sl = list(self._tile_slices(key))
        if arr.split is None or not arr.comm.is_distributed():
            arr.larray[tuple(sl)] = value
            return
        s = arr.split
        counts, displs = arr.counts_displs()
        me = arr.comm.rank
        lo, hi = max(sl[s].start, displs[me]), min(sl[s].stop, displs[me] + counts[me])
        if hi <= lo:
            return
        vsl = [slice(None)] * arr.ndim
        if isinstance(value, torch.Tensor) and value.dim() == arr.ndim:
            vsl[s] = slice(lo - sl[s].start, hi - sl[s].start)
            value = value[tuple(vsl)]
        sl[s] = slice(lo - displs[me], hi - displs[me])
        arr.larray[tuple(sl)] = value


class SquareDiagTiles:
    """Square tiles along the diagonal of a 2-D array (``tiles_per_proc`` tiles per rank along the
    split axis; the other axis reuses the same boundaries)."""

    def __init__(self, arr: DNDarray, tiles_per_proc: int = 2) -> None:
        if not isinstance(arr, DNDarray):
            raise TypeError("arr must be a DNDarray, is currently a {}".format(type(arr)))
        if not isinstance(tiles_per_proc, int):
            raise TypeError("tiles_per_proc must be an int, is currently a {}".format(type(tiles_per_proc)))
        if tiles_per_proc < 1:
            raise ValueError("Tiles per process must be >= 1, currently: {}".format(tiles_per_proc))
        if arr.ndim != 2:
            raise ValueError("Arr must be 2 dimensional, current shape {}".format(arr.shape))
        self.__DNDarray = arr
        self.__lshape_map = arr.create_lshape_map()
        p = arr.comm.size if arr.split is not None else 1
        s = arr.split if arr.split is not None else 0
        counts = self.__lshape_map[:, s].tolist() if arr.split is not None else [arr.gshape[0]]
        rows = []
        tpp = []
        start = 0
        for c in counts:
            k = max(1, min(tiles_per_proc, c)) if c > 0 else 0
            tpp.append(k)
            base, rem = divmod(c, k) if k else (0, 0)
            for t in range(k):
                rows.append(start)
                start += base + (1 if t < rem else 0)
        n_other = arr.gshape[1 - s]
        cols = [r for r in rows if r < n_other] or [0]
        if s == 1:
            rows, cols = cols, rows
        self.__row_inds = [r for r in rows if r < arr.gshape[0]] or [0]
        self.__col_inds = cols if s == 0 else [c for c in cols if c < arr.gshape[1]] or [0]
        self.__tiles_per_proc = tpp
        self.__last_diag_pr = max(0, len([c for c in counts if c > 0]) - 1)

    @property
    def arr(self) -> DNDarray:
        return self.__DNDarray

    @property
    def col_indices(self) -> List[int]:
        return self.__col_inds

    @property
    def row_indices(self) -> List[int]:
        return self.__row_inds

    @property
    def lshape_map(self) -> torch.Tensor:
        return self.__lshape_map

    @property
    def last_diagonal_process(self) -> int:
        return self.__last_diag_pr

    @property
    def tile_columns(self) -> int:
        return len(self.__col_inds)

    @property
    def tile_rows(self) -> int:
        return len(self.__row_inds)

    @property
    def tile_columns_per_process(self) -> List[int]:
        return self.__tiles_per_proc if self.__DNDarray.split == 1 else [self.tile_columns] * len(self.__tiles_per_proc)

    @property
    def tile_rows_per_process(self) -> List[int]:
        return self.__tiles_per_proc if self.__DNDarray.split != 1 else [self.tile_rows] * len(self.__tiles_per_proc)

    @property
    def tile_map(self) -> torch.Tensor:
        """[tile_rows, tile_columns, 3]: (row start, column start, owning rank)."""
        arr = self.__DNDarray
        tm = torch.zeros((self.tile_rows, self.tile_columns, 3), dtype=torch.int64)
        ends = [0] + torch.cumsum(self.__lshape_map[:, arr.split if arr.split is not None else 0], 0).tolist()
        for i, r in enumerate(self.__row_inds):
            for j, c in enumerate(self.__col_inds):
                g = r if arr.split != 1 else c
                owner = 0
                if arr.split is not None:
                    owner = max(q for q in range(len(ends) - 1) if ends[q] <= g)
                tm[i, j] = torch.tensor([r, c, owner])
        return tm

    def get_start_stop(self, key) -> Tuple[int, int, int, int]:
        """Global (row start, row stop, column start, column stop) of tile ``key = (row, col)``."""
        i, j = key
        rows = self.__row_inds + [self.__DNDarray.gshape[0]]
        cols = self.__col_inds + [self.__DNDarray.gshape[1]]
        i = i + self.tile_rows if i < 0 else i
        j = j + self.tile_columns if j < 0 else j
        return rows[i], rows[i + 1], cols[j], cols[j + 1]

    def __getitem__(self, key) -> torch.Tensor:
        arr = self.__DNDarray
        r0, r1, c0, c1 = self.get_start_stop(key)
        if not arr.is_distributed():
            return arr.larray[r0:r1, c0:c1]
        counts, displs = arr.counts_displs()
        me = arr.comm.rank
        lo, hi = displs[me], displs[me] + counts[me]
        if arr.split == 0:
            a, b = max(r0, lo), min(r1, hi)
            return arr.larray[a - lo: b - lo, c0:c1] if b > a else None
        a, b = max(c0, lo), min(c1, hi)
        return arr.larray[r0:r1, a - lo: b - lo] if b > a else None

    def local_get(self, key) -> torch.Tensor:
        return self[key]

    def __setitem__(self, key, value):
        t = self[key]
        if t is not None:
            t[...] = value

    def local_set(self, key, value):
        """Set the part of tile ``key`` (local tile coordinates) this rank holds."""
        self[self.local_to_global(key, self.__DNDarray.comm.rank)] = value

    def local_to_global(self, key, rank: int) -> Tuple[int, int]:
        """Global tile coordinates of the local tile ``key = (row, col)`` of ``rank``: the tile
        index along the split axis is offset by the tiles of the lower ranks."""
        i, j = key
        arr = self.__DNDarray
        if arr.split is None:
            return i, j
        off = sum(self.__tiles_per_proc[:rank])
        return (i + off, j) if arr.split == 0 else (i, j + off)

    def match_tiles(self, tiles_to_match: "SquareDiagTiles") -> None:
        """Adopt the row boundaries of ``tiles_to_match`` (e.g. Q matching R in a tiled QR): the
        rows of this array are cut where the other array's rows are cut."""
        if not isinstance(tiles_to_match, SquareDiagTiles):
            raise TypeError("tiles_to_match must be a SquareDiagTiles, got {}".format(type(tiles_to_match)))
        n = self.__DNDarray.gshape[0]
        rows = [r for r in tiles_to_match.row_indices if r < n] or [0]
        self.__row_inds = rows
        if self.__DNDarray.split == 0:
            ends = [0] + torch.cumsum(self.__lshape_map[:, 0], 0).tolist()
            self.__tiles_per_proc = [len([r for r in rows if ends[q] <= r < ends[q + 1]])
                                     for q in range(len(ends) - 1)]
