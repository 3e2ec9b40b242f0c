"""Synthetic urban scenes for the benchmark configs (SURVEY.md §8(d) scene generator).

uint32 LCG  s <- s*1664525 + 1013904223 (seed 12345); U(a, b) = a + (b - a) * (s >> 8) / 2**24.
Static obstacle: x = U(8, 60), y = U(-20, 20) (|y| < 3 -> y += 6), theta = U(-3.14, 3.14),
size_x = U(2, 6), size_y = U(4, 10), zero velocity.  Moving obstacles are drawn after the static
ones with the same fields (no lane shift) followed by vx = U(-2, 2), vy = U(-2, 2).
The LCG is independent of the planner's rand() stream.
"""
import numpy as np


class _Lcg:
    def __init__(self, seed=12345):
        self.s = seed & 0xFFFFFFFF

    def u(self, a, b):
        self.s = (self.s * 1664525 + 1013904223) & 0xFFFFFFFF
        return a + (b - a) * (self.s >> 8) / 16777216.0


def urban_scene(n_static, n_moving=0, seed=12345):
    """Returns an (M, 7) float64 array of obstacles: cx, cy, theta, size_x, size_y, vx, vy."""
    g = _Lcg(seed)
    out = []
    for _ in range(n_static):
        x = g.u(8.0, 60.0)
        y = g.u(-20.0, 20.0)
        if abs(y) < 3.0:
            y += 6.0
        th = g.u(-3.14, 3.14)
        sx = g.u(2.0, 6.0)
        sy = g.u(4.0, 10.0)
        out.append((x, y, th, sx, sy, 0.0, 0.0))
    for _ in range(n_moving):
        x = g.u(8.0, 60.0)
        y = g.u(-20.0, 20.0)
        th = g.u(-3.14, 3.14)
        sx = g.u(2.0, 6.0)
        sy = g.u(4.0, 10.0)
        vx = g.u(-2.0, 2.0)
        vy = g.u(-2.0, 2.0)
        out.append((x, y, th, sx, sy, vx, vy))
    return np.asarray(out, dtype=np.float64).reshape(-1, 7)
