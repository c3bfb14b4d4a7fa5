"""Pure-Python restatement of Game2048.step (game.py:923-1030).  TEST / BASELINE INFRASTRUCTURE ONLY.

Used (a) as a second, independent checker of the golden games and (b) by bench.py's cpu_baseline
leg to time "the reference's CPU path" on the GPU box, where the reference itself is not present.
It keeps the reference's per-step cost structure: Python ints in lists, the global `random`
module for spawns (random.choice / random.random, game.py:937-939), and all 17 heuristic
evaluations that game.step performs before/after every move (game.py:981-1002), although only
monotonicity and emptiness feed the reward.  Boards are flat 16-lists (cell 4*i+j).
"""

from __future__ import annotations

import random
import time

_CORNERS = (0, 3, 12, 15)
_NEIGH = [[q for q in ((p - 4) if p >= 4 else None, (p + 4) if p < 12 else None,
                       (p - 1) if p % 4 else None, (p + 1) if p % 4 != 3 else None) if q is not None]
          for p in range(16)]
# (dir -> the 4 lines of cell indices, ordered from the edge the tiles slide toward) game.py:122-160
_LINES = {
    0: [[c, c + 4, c + 8, c + 12] for c in range(4)],          # UP
    1: [[c + 12, c + 8, c + 4, c] for c in range(4)],          # DOWN
    2: [[4 * r, 4 * r + 1, 4 * r + 2, 4 * r + 3] for r in range(4)],  # LEFT
    3: [[4 * r + 3, 4 * r + 2, 4 * r + 1, 4 * r] for r in range(4)],  # RIGHT
}


def slide(b, d):
    """simulate_move: returns (new board, points, max tile created)."""
    out = [0] * 16
    pts = mx = 0
    for line in _LINES[d]:
        vals = [b[p] for p in line if b[p]]
        k = i = 0
        while i < len(vals):
            if i + 1 < len(vals) and vals[i] == vals[i + 1]:
                e = vals[i] + 1
                out[line[k]] = e
                pts += 1 << e
                mx = max(mx, e)
                i += 2
            else:
                out[line[k]] = vals[i]
                i += 1
            k += 1
    return out, pts, mx


def legal_mask(b) -> int:
    return sum(1 << d for d in range(4) if slide(b, d)[0] != b)


def emptiness(b) -> int:
    return b.count(0)


def monotonicity(b) -> int:
    g = b
    best = -1
    for _ in range(4):
        c = 0
        for i in range(4):
            for j in range(3):
                x, y = g[4 * i + j], g[4 * i + j + 1]
                if x and y and x >= y:
                    c += 1
        for j in range(4):
            for i in range(3):
                x, y = g[4 * i + j], g[4 * i + 4 + j]
                if x and y and x >= y:
                    c += 1
        best = max(best, c)
        g = [g[4 * (3 - j) + i] for i in range(4) for j in range(4)]
    m = max(b)
    pos = b.index(m)
    return best * 2 if pos in _CORNERS else best // 2


def smoothness(b) -> float:
    s = 0.0
    for p in range(16):
        if b[p]:
            if p % 4 != 3 and b[p + 1]:
                s -= abs(b[p] - b[p + 1])
            if p < 12 and b[p + 4]:
                s -= abs(b[p] - b[p + 4])
    return s


def corner_bonus(b) -> float:
    m = max(b)
    if m == 0:
        return 0.0
    return float(m) if any(b[c] == m for c in _CORNERS) else -float(m)


def adjacency(b) -> float:
    m, mp = 0, 0
    for p in range(16):
        if b[p] > m:
            m, mp = b[p], p
    bonus = 0.0
    for q in _NEIGH_ORDERED[mp]:
        if q is not None and b[q] > 0:
            bonus += b[q] * 0.5
    for p in range(16):
        if b[p] >= 5:
            if p % 4 != 3 and b[p + 1] >= 5:
                bonus += (b[p] + b[p + 1]) * 0.25
            if p < 12 and b[p + 4] >= 5:
                bonus += (b[p] + b[p + 4]) * 0.25
    return bonus


def chain(b) -> float:
    m = max(b)
    if m == 0:
        return 0.0

    def walk(p, want, seen):
        if p in seen or b[p] != want:
            return 0.0
        seen.add(p)
        best = 0.0
        for q in _NEIGH_ORDERED[p]:
            if q is not None:
                best = max(best, walk(q, want - 1, seen))
        seen.discard(p)
        return float(want) + best

    return max(walk(p, m, set()) for p in range(16) if b[p] == m)


# neighbour order of the reference DFS: up, down, left, right (None = off-board)
_NEIGH_ORDERED = [((p - 4) if p >= 4 else None, (p + 4) if p < 12 else None,
                   (p - 1) if p % 4 else None, (p + 1) if p % 4 != 3 else None) for p in range(16)]


def anchor(b) -> int:
    m = max(b)
    if m == 0:
        return 0
    tops = [p for p in range(16) if b[p] == m]
    for p in tops:
        if p in _CORNERS:
            return p
    t = tops[0]
    return min(_CORNERS, key=lambda c: abs(c // 4 - t // 4) + abs(c % 4 - t % 4))


def _snake(corner):
    r0, c0 = divmod(corner, 4)
    dr, dc = (1 if r0 == 0 else -1), (1 if c0 == 0 else -1)
    order = []
    for i in range(4):
        cols = [c0 + s * dc for s in range(4)]
        if i % 2:
            cols.reverse()
        order += [4 * (r0 + i * dr) + c for c in cols]
    return order


_SNAKES = {c: _snake(c) for c in _CORNERS}


def topological(b, corner) -> float:
    tiles = [(b[p], p) for p in range(16) if b[p] > 0]
    if not tiles:
        return 0.0
    m = max(v for v, _ in tiles)
    order = _SNAKES[corner]
    idx = {p: k for k, p in enumerate(order)}
    score = 0.0
    for v, p in tiles:
        score += (16 - idx[p]) * v * 0.1
    prev = float("inf")
    mono = inv = 0.0
    for p in order:
        v = b[p]
        if v == 0:
            continue
        if v <= prev:
            mono += v * 0.2
        else:
            inv += (v - prev) * 0.5
        prev = v
    score += mono - inv
    if b[corner] == m:
        score += m * 2.0
    for v, p in tiles:
        if v < 4:
            continue
        nb = [b[q] for q in _NEIGH[p] if b[q] > 0]
        lower = sum(1 for x in nb if x < v - 2)
        if len(nb) >= 2 and lower >= len(nb) - 1 and idx[p] > 4:
            score -= v * 1.0
    return score


def add_tile(b, rnd=random):
    empties = [p for p in range(16) if b[p] == 0]
    if not empties:
        return False
    p = rnd.choice(empties)
    b[p] = 1 if rnd.random() < 0.9 else 2
    return True


def reset(rnd=random):
    b = [0] * 16
    add_tile(b, rnd)
    add_tile(b, rnd)
    return b


def step(b, d, rnd=random):
    """Game2048.step on flat board `b` (mutated).  Returns (points, done, info dict)."""
    new, pts, mx = slide(b, d)
    if new == b:
        return 0, legal_mask(b) == 0, {"invalid_move": True, "monotonicity_before": 0.0,
                                       "monotonicity_after": 0.0, "emptiness_before": 0.0,
                                       "emptiness_after": 0.0, "max_tile_created": 0}
    sb, cb, ab, chb = smoothness(b), corner_bonus(b), adjacency(b), chain(b)
    mb = monotonicity(b)
    anc = anchor(b)
    tb = topological(b, anc)
    eb = emptiness(b)
    xb = max(b)
    b[:] = new
    info = {"invalid_move": False, "smoothness_delta": smoothness(b) - sb, "corner_delta": corner_bonus(b) - cb,
            "adjacency_delta": adjacency(b) - ab, "chain_delta": chain(b) - chb,
            "monotonicity_before": mb, "monotonicity_after": monotonicity(b),
            "emptiness_before": eb, "emptiness_after": emptiness(b),
            "topological_delta": topological(b, anc) - tb, "max_tile_created": mx,
            "max_exponent_before": xb, "max_exponent_after": max(b), "topological_anchor": anc}
    add_tile(b, rnd)
    return pts, legal_mask(b) == 0, info


def time_random_steps(seconds: float, seed: int = 0x2048) -> dict:
    """Random-legal-action game loop with auto-reset, the reference's per-step cost (1 core)."""
    rnd = random.Random(seed)
    b = reset(rnd)
    n = 0
    t0 = time.perf_counter()
    deadline = t0 + seconds
    while True:
        for _ in range(200):
            legal_dirs = [d for d in range(4) if slide(b, d)[0] != b]
            _, done, _ = step(b, rnd.choice(legal_dirs), rnd)
            n += 1
            if done:
                b = reset(rnd)
        if time.perf_counter() >= deadline:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "steps": n, "seconds": dt,
            "sample": f"{n} random-legal game.step calls (pure-Python restatement incl. 17 heuristic "
                      f"evaluations per step), 1 core, {dt:.1f} s"}
