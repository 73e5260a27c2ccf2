"""cfg5 (BASELINE configs[4]: 10 views at 6048x4032, "tiled per-image,
2 GPUs") on one MI355X: the unsplit RunPatchMatch against each of its two row
bands run alone (acmmp_run_patchmatch_band, 23-row halo of
src/ACMMP.cu:819-826).

A band run alone is the per-GPU compute of the 2-GPU split. Its halo
callback only synchronises the engine stream, as the real exchange does
before it ships the rows (acmmp_amd/band.py), so the host round trip after
every half-sweep is inside the timing; the rows themselves (2 x 23 rows x
3024 colour-split pixels x 24 B = 3.3 MB per half-sweep) and the final band
all-gather (0.24 GB) are priced at 100 GB/s of xGMI and added as a model
(not measured: this box has one GPU). Timings are medians of `reps` after
one warm-up, inputs resident in HBM.

usage: python tools/cfg5_band_timing.py [reps] > gpurun_out/cfg5_bands.json
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from acmmp_amd import ACMMP, default_params, scene  # noqa: E402
from acmmp_amd.band import bands  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
W, H, NSRC, ITERS = 6048, 4032, 9, 8
XGMI_GBS = 100.0
dev = torch.device("cuda", 0)


def _timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    setup = scene.scene_setup(num_views=NSRC + 1, width=W, height=H)
    ids = [0] + list(setup.pairs[0][:NSRC])
    imgs = [scene.render_torch(setup, i, dev) for i in ids]
    torch.cuda.synchronize()
    cams = [setup.camera(i) for i in ids]
    out = {"config": "cfg5", "W": W, "H": H, "num_images": NSRC + 1, "iters": ITERS, "reps": REPS}
    with ACMMP(0) as eng:
        p = default_params()
        p.max_iterations = ITERS
        eng.set_params(p)
        eng.set_images_device(cams, [im.data_ptr() for im in imgs])
        ms = [_timed(eng.RunPatchMatch) for _ in range(REPS + 1)][1:]
        out["unsplit_ms"] = statistics.median(ms)
        halves = bands(H, 2)
        syncs = [0]

        def local(halo):  # what TorchBandExchange does before it ships the rows
            torch.cuda.ExternalStream(int(halo.stream), device=dev).synchronize()
            syncs[0] += 1

        band_ms = []
        for lo, hi in halves:
            ms = [_timed(lambda: eng.run_band(lo, hi, local)) for _ in range(REPS + 1)][1:]
            band_ms.append(statistics.median(ms))
        out["bands"] = [list(b) for b in halves]
        out["band_ms"] = band_ms
        out["half_sweeps"] = syncs[0] // (REPS + 1) // 2
    halo_bytes = 2 * 23 * ((W + 1) // 2) * 24
    gather_bytes = (H // 2) * W * 20
    model_ms = out["half_sweeps"] * halo_bytes / (XGMI_GBS * 1e9) * 1e3 + gather_bytes / (XGMI_GBS * 1e9) * 1e3
    out["xgmi_model_ms"] = model_ms
    out["two_gpu_estimate_ms"] = max(band_ms) + model_ms
    out["speedup_estimate"] = out["unsplit_ms"] / out["two_gpu_estimate_ms"]
    out["unsplit_mpix_s"] = W * H / out["unsplit_ms"] / 1e3
    out["two_gpu_estimate_mpix_s"] = W * H / out["two_gpu_estimate_ms"] / 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
