"""Run the same RunPatchMatch several times (fresh engines, with other work in
between: a scribble over freed device memory, or a run at another size) and
report whether the outputs are bitwise identical."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from acmmp_amd import ACMMP, default_params, scene

W = int(sys.argv[1]) if len(sys.argv) > 1 else 6048
H = int(sys.argv[2]) if len(sys.argv) > 2 else 4032
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
dev = torch.device("cuda", 0)


def problem(w, h):
    setup = scene.scene_setup(num_views=10, width=w, height=h)
    ids = [0] + list(setup.pairs[0][:9])
    imgs = [scene.render_torch(setup, i, dev) for i in ids]
    torch.cuda.synchronize()
    return [setup.camera(i) for i in ids], imgs


def run(cams, imgs):
    with ACMMP(0) as eng:
        p = default_params(); p.max_iterations = iters
        eng.set_params(p)
        eng.set_images_device(cams, [im.data_ptr() for im in imgs])
        eng.RunPatchMatch()
        return eng.plane_hypotheses(), eng.costs()


cams, imgs = problem(W, H)
outs = [run(cams, imgs)]
x = torch.full((W * H * 40,), float("nan"), device=dev)
del x
torch.cuda.empty_cache()
outs.append(run(cams, imgs))
c2, i2 = problem(1600, 1200)
run(c2, i2)
del i2
outs.append(run(cams, imgs))
del imgs
cams, imgs = problem(W, H)  # fresh allocations
outs.append(run(cams, imgs))
for k in range(1, len(outs)):
    dp = (outs[k][0].view(np.uint32) != outs[0][0].view(np.uint32)).any(-1)
    dc = (outs[k][1].view(np.uint32) != outs[0][1].view(np.uint32)) & ~(np.isnan(outs[k][1]) & np.isnan(outs[0][1]))
    rows = np.nonzero(dp.any(1))[0]
    print(json.dumps({"W": W, "H": H, "run": k, "plane_diff_px": int(dp.sum()), "cost_diff_px": int(dc.sum()),
                      "first_rows": rows[:10].tolist(), "finite": [float(np.isfinite(o[1]).mean()) for o in outs]}),
          flush=True)
