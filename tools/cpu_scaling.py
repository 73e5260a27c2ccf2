"""OpenMP scaling of the CPU baseline (oracle/acmmp_oracle.c), so the bench
line's all-core estimate rests on a measured parallel efficiency rather than
on linearity alone. Times bench.py's cpu_baseline work —
a crop of cfg2's reference view 0 (principal point shifted) against its 9
full 1600x1200 source views, photometric, 8 iterations — at 1, 2, 4, ... host
threads and prints one JSON line per thread count plus the efficiencies.

usage: python tools/cpu_scaling.py [crop WxH] [max threads]   (CPU only)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (test infrastructure: the CPU baseline itself)
from acmmp_amd import default_params, scene  # noqa: E402
from acmmp_amd._abi import Camera  # noqa: E402


def main():
    cw, ch = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "400x300").split("x"))
    tmax = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    W, H = 1600, 1200
    setup = scene.scene_setup(num_views=10, width=W, height=H)
    ids = [0] + list(setup.pairs[0][:9])
    imgs = [scene.render_numpy(setup, i).image.astype(np.float32) for i in ids]
    cams = [setup.camera(i) for i in ids]
    x0, y0 = (W - cw) // 2, (H - ch) // 2
    ref = Camera.from_buffer_copy(bytes(cams[0]))
    ref.K[2] = cams[0].K[2] - x0
    ref.K[5] = cams[0].K[5] - y0
    ref.width, ref.height = cw, ch
    imgs[0] = np.ascontiguousarray(imgs[0][y0:y0 + ch, x0:x0 + cw])
    cams = [ref] + cams[1:]
    p = default_params()
    p.max_iterations = 8
    p.depth_min = cams[0].depth_min * 0.6
    p.depth_max = cams[0].depth_max * 1.2
    oracle.build()
    rows, t = [], 1
    while t <= tmax:
        t0 = time.perf_counter()
        oracle.run_patchmatch(p, cams, imgs, nthreads=t)
        dt = time.perf_counter() - t0
        rows.append({"threads": t, "seconds": round(dt, 3), "mpix_s": round(cw * ch / dt / 1e6, 6)})
        print(json.dumps(rows[-1]), flush=True)
        t *= 2
    base = rows[0]["mpix_s"]
    print(json.dumps({"crop": f"{cw}x{ch}", "cpu_count": os.cpu_count(),
                      "efficiency": {r["threads"]: round(r["mpix_s"] / (base * r["threads"]), 3) for r in rows}}))


if __name__ == "__main__":
    main()
