"""Job-list helpers shared by the entropy tests: the quadtree walk and the
coefficient distribution of tools/refeval/gen_ec_ref.py (no reference text
involved: only the shapes the vectors use)."""
import numpy as np


def rand_coeffs(rng, cw, scale):
    if rng.random() < 0.15:
        return np.zeros(cw * cw, np.int64)
    r = np.arange(cw)
    decay = np.exp(-(r[:, None] + r[None, :]) / (cw * rng.uniform(0.05, 0.6)))
    c = np.round(rng.laplace(0, scale, (cw, cw)) * decay).astype(np.int64)
    if rng.random() < 0.3:
        for _ in range(int(rng.integers(1, 4))):
            c[int(rng.integers(0, min(cw, 6))), int(rng.integers(0, min(cw, 6)))] = int(
                rng.integers(-3000, 3000))
    if rng.random() < 0.2:
        c[np.abs(c) < 3] = 0
    return c.reshape(-1)


def leaves(rng, x4, y4, lg, minlg, vis_w4, vis_h4, out):
    if x4 >= vis_w4 or y4 >= vis_h4:
        return
    n4 = 1 << (lg - 2)
    must = x4 + n4 > vis_w4 or y4 + n4 > vis_h4
    if lg > minlg and (must or rng.random() < 0.45):
        h = n4 // 2
        for dy in (0, h):
            for dx in (0, h):
                leaves(rng, x4 + dx, y4 + dy, lg - 1, minlg, vis_w4, vis_h4, out)
    else:
        out.append((x4, y4, lg))
