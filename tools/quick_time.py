"""Single-view GPU timing probe: one RunPatchMatch at WxH with N images."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from acmmp_amd import ACMMP, default_params, scene

W = int(sys.argv[1]) if len(sys.argv) > 1 else 1600
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
nimg = int(sys.argv[4]) if len(sys.argv) > 4 else 10
dev = torch.device("cuda", 0)
setup = scene.scene_setup(num_views=nimg, width=W, height=H)
ids = [0] + setup.pairs[0][:nimg - 1]
imgs = [scene.render_torch(setup, i, dev) for i in ids]
torch.cuda.synchronize()
eng = ACMMP(0)
eng.set_timing(True)
p = default_params(); p.max_iterations = iters
eng.set_params(p)
eng.set_images_device([setup.camera(i) for i in ids], [im.data_ptr() for im in imgs])
for rep in range(3):
    t0 = time.perf_counter(); eng.RunPatchMatch(); dt = time.perf_counter() - t0
    t = eng.timing(); t["launch_ms"] = t["sweep_ms"] / max(t["sweep_launches"], 1)
    print(json.dumps({"lib": os.environ.get("ACMMP_LIB", "default"), "W": W, "H": H, "iters": iters, "nimg": nimg, "wall_ms": dt * 1e3, **t}), flush=True)
co = eng.costs()
print("cost<0.5 frac", float((co < 0.5).mean()))
