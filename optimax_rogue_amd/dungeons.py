"""DungeonBank: an explicit-grid DungeonGenerator plugin for the engine.

The reference's generator API is ``DungeonGenerator(width, height)
.spawn_dungeon(depth) -> Dungeon(tiles)`` (optimax_rogue/logic/worldgen.py:9-26);
arbitrary Python cannot run inside the tick kernel, so the batched form of an
explicit-grid generator is data: a bank of L layouts (``Dungeon.tiles``
arrays, Tile codes Ground 1 / Wall 2 / StaircaseDown 3, world.py:10-17) from
which ``spawn_dungeon`` picks ``np.random.randint(L)``.  Everything the updater
asks of a dungeon is then precomputed per layout:

* ``is_blocked`` (world.py:41-46): the tiles themselves (bank_tiles),
* ``get_random_unblocked`` (world.py:57-66): the flat indices x * H + y of
  the Ground tiles in ascending order (bank_ground) -- the c-th Ground tile is
  one load instead of a W x H scan,
* ``staircase`` (world.py:52-55): the first StaircaseDown in x-major order
  (bank_meta), what StaircaseBot walks to; stepping on ANY StaircaseDown tile
  descends (updater.py:205-206).
"""
from __future__ import annotations

import numpy as np

from .enums import Tile


class DungeonBank:
    """L layouts of one width x height; validates them like the reference would
    fail on them (no staircase: ``Dungeon.staircase`` raises IndexError)."""

    def __init__(self, layouts):
        a = np.asarray(layouts)
        if a.ndim == 2:
            a = a[None]
        if a.ndim != 3 or a.shape[0] < 1:
            raise ValueError("layouts must be [L, W, H] Tile codes")
        if not np.isin(a, [Tile.Ground, Tile.Wall, Tile.StaircaseDown]).all():
            raise ValueError("layout tiles must be Ground (1), Wall (2) or StaircaseDown (3)")
        L, W, H = a.shape
        if L > 32767 or W * H > 65536:
            raise ValueError("a bank holds at most 32767 layouts of at most 65536 tiles")
        self.layouts = np.ascontiguousarray(a, np.uint8)
        self.width, self.height = int(W), int(H)
        flat = self.layouts.reshape(L, W * H)
        self.ground = np.zeros((L, W * H), np.uint16)
        self.meta = np.zeros((L, 4), np.int32)
        for li in range(L):
            g = np.flatnonzero(flat[li] == Tile.Ground)
            st = np.flatnonzero(flat[li] == Tile.StaircaseDown)
            if len(st) == 0:
                raise ValueError(f"layout {li} has no StaircaseDown tile")
            self.ground[li, :len(g)] = g
            self.meta[li] = (len(g), st[0] // H, st[0] % H, 0)

    @classmethod
    def random(cls, width: int, height: int, n_layouts: int, seed: int = 0,
               wall_p: float = 0.15, n_stairs: int = 1) -> "DungeonBank":
        """A synthetic bank: border walls, interior walls with probability
        ``wall_p``, ``n_stairs`` staircases on Ground tiles (numpy
        RandomState(seed); connectivity is not required by the updater)."""
        rs = np.random.RandomState(seed)
        out = []
        for _ in range(int(n_layouts)):
            t = np.full((width, height), Tile.Ground, np.uint8)
            t[[0, -1], :] = Tile.Wall
            t[:, [0, -1]] = Tile.Wall
            inner = rs.rand(width, height) < wall_p
            inner[[0, -1], :] = False
            inner[:, [0, -1]] = False
            t[inner] = Tile.Wall
            ground = np.argwhere(t == Tile.Ground)
            for j in rs.choice(len(ground), n_stairs, replace=False):
                t[tuple(ground[j])] = Tile.StaircaseDown
            out.append(t)
        return cls(np.stack(out))

    def __len__(self) -> int:
        return len(self.layouts)

    @property
    def min_ground(self) -> int:
        return int(self.meta[:, 0].min())

    def staircase(self, layout: int):
        return int(self.meta[layout, 1]), int(self.meta[layout, 2])

    def tiles(self, layout: int) -> np.ndarray:
        """Dungeon.tiles of a layout as the reference stores them (int32)."""
        return self.layouts[layout].astype(np.int32)

    def spawn_dungeon(self, depth: int):
        """The generator on the CPU with numpy's global RandomState, as a
        reference DungeonGenerator would run: (layout index, tiles)."""
        i = int(np.random.randint(len(self.layouts)))
        return i, self.tiles(i)
