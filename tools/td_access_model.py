"""Predicted TCP accesses per k_sweep gather for each lane map, from the
access rule measured in profiles/r04_td_addressing.md §2: one access per
distinct 64-B line per group of 8 lanes, a group being the even or the odd
lanes of one 16-lane quarter of the wave (fits all 12 td_rule patterns; a
quarter reading one contiguous 64-B line costs 1 in total).

Sample positions: the synthetic cfg2 scene at its analytic depth (converged
planes): every colour-c pixel's 36 patch samples (offsets -5..5 step 2)
projected into its nearest source view; records of the u8-quad form (4 B,
row pitch as the engine pads it); waves of 8 x 8 colour-split pixels.

usage: python tools/td_access_model.py [width height]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acmmp_amd import scene  # noqa: E402

MAPS = {
    0: lambda l: (l % 8, l // 8),
    1: lambda l: ((l & 3) + 4 * ((l >> 4) & 1), ((l >> 2) & 3) + 4 * (l >> 5)),
    2: lambda l: (((l >> 2) & 3) + 4 * ((l >> 4) & 1), (l & 3) + 4 * (l >> 5)),
    3: lambda l: ((l >> 1) & 7, (l & 1) + 2 * (l >> 4)),
}


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    setup = scene.scene_setup(num_views=3, width=W, height=H)
    ref = scene.render_numpy(setup, 0)
    src = setup.pairs[0][0]
    Rs, ts, _, _ = setup.poses[src]
    R0, t0 = ref.R.astype(np.float64), ref.t.astype(np.float64)
    K = setup.K
    pitch = (W + 3 + 15) // 16 * 16
    ys, xs = np.mgrid[0:H, 0:W]
    d = ref.depth.astype(np.float64)
    # world point of every ref pixel, projected into the source view
    cam = np.stack([(xs - K[0, 2]) / K[0, 0] * d, (ys - K[1, 2]) / K[1, 1] * d, d], -1)
    Xw = (cam - t0) @ R0  # R^T (x - t)
    xs_c = Xw @ Rs.T + ts
    u = K[0, 0] * xs_c[..., 0] / xs_c[..., 2] + K[0, 2]
    v = K[1, 1] * xs_c[..., 1] / xs_c[..., 2] + K[1, 2]
    ok = d > 0
    rec = (np.clip(np.floor(v), -1, H) + 1) * pitch + np.clip(np.floor(u), -1, W) + 1
    rec = np.where(ok, rec, -1).astype(np.int64)
    offs = [(i, j) for j in range(-5, 6, 2) for i in range(-5, 6, 2)]
    Wh = W // 2
    res = {}
    for m, f in MAPS.items():
        lc, lr = np.array([f(l) for l in range(64)]).T
        total = cnt = 0
        for colour in (0, 1):
            for wy in range(8, H - 16, 24):
                for wk in range(4, Wh - 12, 24):
                    py = wy + lr
                    px = 2 * (wk + lc) + ((py + colour) & 1)
                    for (i, j) in offs[::3]:
                        r = rec[py + j, px + i]
                        if (r < 0).any():
                            continue
                        lines = (r * 4) // 64
                        acc = 0
                        for q in range(4):
                            for par in range(2):
                                acc += len(np.unique(lines[q * 16 + par::2][:8]))
                        total += acc
                        cnt += 1
        res[m] = total / max(cnt, 1)
        print(f"lane map {m}: {res[m]:.2f} predicted accesses per gather ({cnt} gathers)")


if __name__ == "__main__":
    main()
