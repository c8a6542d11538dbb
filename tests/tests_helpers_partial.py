"""Small host helpers shared by the MARL_PARTIAL tests."""
import numpy as np


def largest_component(g):
    """Cells outside the largest 4-connected free component become obstacles."""
    s0, s1 = g.shape
    seen = np.zeros(g.shape, dtype=bool)
    best = []
    for r in range(s0):
        for c in range(s1):
            if g[r, c] == 0 and not seen[r, c]:
                comp, stack = [], [(r, c)]
                seen[r, c] = True
                while stack:
                    y, x = stack.pop()
                    comp.append((y, x))
                    for dy, dx in ((1, 0), (-1, 0), (0, 1), (0, -1)):
                        yy, xx = y + dy, x + dx
                        if 0 <= yy < s0 and 0 <= xx < s1 and g[yy, xx] == 0 and not seen[yy, xx]:
                            seen[yy, xx] = True
                            stack.append((yy, xx))
                if len(comp) > len(best):
                    best = comp
    out = np.full_like(g, -1)
    for y, x in best:
        out[y, x] = 0
    return out
