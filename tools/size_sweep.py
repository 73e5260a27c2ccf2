import os, sys, json
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from acmmp_amd import ACMMP, default_params, scene
dev = torch.device("cuda", 0)
for (W, H, wide) in [(1600, 1200, 0), (1600, 1200, 1), (3200, 2133, 0), (3200, 2133, 1), (6048, 4032, 0)]:
    os.environ["ACMMP_WIDE_INDEX"] = str(wide)
    setup = scene.scene_setup(num_views=10, width=W, height=H)
    ids = [0] + list(setup.pairs[0][:9])
    imgs = [scene.render_torch(setup, i, dev) for i in ids]
    img0, gt = scene.render_torch(setup, 0, dev, with_depth=True)
    torch.cuda.synchronize()
    with ACMMP(0) as eng:
        p = default_params(); p.max_iterations = 8
        eng.set_params(p)
        eng.set_images_device([setup.camera(i) for i in ids], [im.data_ptr() for im in imgs])
        eng.RunPatchMatch()
        pl, co = eng.plane_hypotheses(), eng.costs()
    gt = gt.cpu().numpy(); im = img0.cpu().numpy()
    hit = gt > 0
    print(json.dumps({"W": W, "H": H, "wide": wide, "finite": float(np.isfinite(co).mean()),
                      "finite_on_hit": float(np.isfinite(co)[hit].mean()), "hit": float(hit.mean()),
                      "flat128": float((im == 128).mean()), "cost<0.5": float((co < 0.5).mean()),
                      "rows_nan_frac": [float(np.isnan(co[r]).mean()) for r in range(0, H, H // 8)]}), flush=True)
