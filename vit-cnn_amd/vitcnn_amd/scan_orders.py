"""Token orders of hsiMamba's 10 scan directions, generated from their rules.

The reference stores them as literal tables for n = 9 ('81_2+8', Mutimodality_Mamba7.py:609-640)
and n = 7 ('49_2+8', :788-806) and derives the reverses with torch.flip (:614, :620, :626, :643).
Gate order (:653, :699-701): hf, hr, vf, vr, 37df, 37dr, 19df, 19dr, ltcw, ltacw.
Rules (pinned against the reference tables in tests/test_host_logic.py):
  hf    row-major identity               hr   its reverse
  vf    column snake (down, up, down...) vr   its reverse
  37df  anti-diagonal zigzag from (0,0)  37dr its reverse
  19df  the same zigzag mirrored L<->R   19dr its reverse
  ltcw  clockwise spiral from top-left   ltacw anticlockwise spiral from top-left
For other n (the documented generalisation, SURVEY.md section 8 row A-MUUFL) the same rules apply.
"""
from __future__ import annotations

from typing import List


def _column_snake(n: int) -> List[int]:
    seq = []
    for col in range(n):
        rows = range(n) if col % 2 == 0 else reversed(range(n))
        seq.extend(r * n + col for r in rows)
    return seq


def _antidiagonal_zigzag(n: int, mirrored: bool) -> List[int]:
    seq = []
    for diag in range(2 * n - 1):
        lo, hi = max(0, diag - n + 1), min(diag, n - 1)
        rows = list(range(lo, hi + 1))
        if diag % 2 == 0:
            rows.reverse()
        for r in rows:
            c = diag - r
            seq.append(r * n + ((n - 1 - c) if mirrored else c))
    return seq


def _spiral(n: int, clockwise: bool) -> List[int]:
    seen = [[False] * n for _ in range(n)]
    # clockwise: right, down, left, up ; anticlockwise: down, right, up, left
    moves = [(0, 1), (1, 0), (0, -1), (-1, 0)] if clockwise else [(1, 0), (0, 1), (-1, 0), (0, -1)]
    r = c = k = 0
    seq = []
    for _ in range(n * n):
        seq.append(r * n + c)
        seen[r][c] = True
        dr, dc = moves[k]
        nr, nc = r + dr, c + dc
        if not (0 <= nr < n and 0 <= nc < n) or seen[nr][nc]:
            k = (k + 1) % 4
            dr, dc = moves[k]
            nr, nc = r + dr, c + dc
        r, c = nr, nc
    return seq


def scan_orders(n: int) -> List[List[int]]:
    """10 orders for an n x n token grid: order[k][t] = token at sequence position t."""
    hf = list(range(n * n))
    vf = _column_snake(n)
    d37 = _antidiagonal_zigzag(n, mirrored=False)
    d19 = _antidiagonal_zigzag(n, mirrored=True)
    return [hf, hf[::-1], vf, vf[::-1], d37, d37[::-1], d19, d19[::-1], _spiral(n, True), _spiral(n, False)]


def inverse(order: List[int]) -> List[int]:
    inv = [0] * len(order)
    for pos, tok in enumerate(order):
        inv[tok] = pos
    return inv
