"""Map data for the marl-delivery grid world.

The ``map*.txt`` files are the reference's own maps (data, whitespace-separated
0/1 grids; ``/root/reference/map*.txt``).  ``load_map`` follows the reference
parser ``Environment.load_map`` (``env.py:45-57``): one row per line,
``line.strip().split(' ')``, ``int()`` per token.

``synthetic_map`` builds the 64x64 stress map of BASELINE.json config 5
(border walls, ~10 % interior obstacles, seed 7, free region made connected).
"""
from __future__ import annotations

import os
from collections import deque

import numpy as np

MAP_DIR = os.path.dirname(os.path.abspath(__file__))
BUILTIN = ("map.txt", "map1.txt", "map2.txt", "map3.txt", "map4.txt", "map5.txt")


def map_path(name: str) -> str:
    """Resolve a builtin map name (``"map1"`` / ``"map1.txt"``) or return ``name``."""
    if os.path.exists(name):
        return name
    cand = name if name.endswith(".txt") else name + ".txt"
    p = os.path.join(MAP_DIR, os.path.basename(cand))
    if os.path.exists(p):
        return p
    raise FileNotFoundError(name)


def load_map(path: str) -> list[list[int]]:
    """Parse a map file exactly like ``env.py:45-57`` (raises on the same inputs)."""
    grid = []
    with open(path, "r") as f:
        for line in f:
            grid.append([int(x) for x in line.strip().split(" ")])
    return grid


def grid_array(grid) -> np.ndarray:
    g = np.asarray(grid, dtype=np.uint8)
    if g.ndim != 2:
        raise ValueError("map must be rectangular")
    return np.ascontiguousarray(g)


def synthetic_map(h: int = 64, w: int = 64, density: float = 0.10, seed: int = 7) -> np.ndarray:
    """Border walls + random interior obstacles; unreachable free cells are walled in."""
    rs = np.random.RandomState(seed)
    g = (rs.random_sample((h, w)) < density).astype(np.uint8)
    g[0, :] = 1
    g[-1, :] = 1
    g[:, 0] = 1
    g[:, -1] = 1
    free = np.argwhere(g == 0)
    seen = np.zeros_like(g, dtype=bool)
    # keep the largest 4-connected free component
    best = None
    for r0, c0 in free:
        if seen[r0, c0]:
            continue
        comp = []
        dq = deque([(r0, c0)])
        seen[r0, c0] = True
        while dq:
            r, c = dq.popleft()
            comp.append((r, c))
            for dr, dc in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                rr, cc = r + dr, c + dc
                if 0 <= rr < h and 0 <= cc < w and not seen[rr, cc] and g[rr, cc] == 0:
                    seen[rr, cc] = True
                    dq.append((rr, cc))
        if best is None or len(comp) > len(best):
            best = comp
    out = np.ones_like(g)
    for r, c in best:
        out[r, c] = 0
    return out


def write_map(path: str, grid) -> None:
    g = grid_array(grid)
    with open(path, "w") as f:
        f.write("\n".join(" ".join(str(int(v)) for v in row) for row in g))
        f.write("\n")
