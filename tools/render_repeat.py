"""render_torch determinism (repeat calls) and agreement with render_numpy."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from acmmp_amd import scene

dev = torch.device("cuda", 0)
for (W, H) in [(320, 240), (1600, 1200), (6048, 4032)]:
    setup = scene.scene_setup(num_views=10, width=W, height=H)
    a = [scene.render_torch(setup, i, dev) for i in range(3)]
    b = [scene.render_torch(setup, i, dev) for i in range(3)]
    line = f"{W}x{H} repeat-diff {[int((x != y).sum()) for x, y in zip(a, b)]}"
    if W * H <= 2_000_000:
        v = scene.render_numpy(setup, 0)
        img, z = scene.render_torch(setup, 0, dev, with_depth=True)
        line += f" numpy-diff img {int((img.cpu().numpy() != v.image).sum())} depth max rel " \
                f"{float(np.max(np.abs(z.cpu().numpy() - v.depth) / np.maximum(v.depth, 1))):.2e}"
    print(line, flush=True)
