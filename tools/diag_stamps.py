"""Phase split of k_sweep from an ACMMP_DIAG_STAMPS build (diagnostic only).
usage: ACMMP_LIB=acmmp_amd/lib/variants/libacmmp_amd_diag.so python tools/diag_stamps.py"""
import ctypes as C, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from acmmp_amd import ACMMP, default_params, scene, _abi
lib = _abi.load_library()
fn = lib.acmmp_diag_read_cycles
fn.restype = C.c_int; fn.argtypes = [C.POINTER(C.c_uint64)]
dev = torch.device("cuda", 0)
setup = scene.scene_setup(num_views=10, width=1600, height=1200)
ids = [0] + setup.pairs[0][:9]
imgs = [scene.render_torch(setup, i, dev) for i in ids]
eng = ACMMP(0); p = default_params(); p.max_iterations = 8; eng.set_params(p)
eng.set_images_device([setup.camera(i) for i in ids], [im.data_ptr() for im in imgs])
eng.RunPatchMatch()
out = (C.c_uint64 * 24)(); fn(out)  # reset after warmup
eng.RunPatchMatch()
fn(out)
names = ["tile+search", "pixel_patch", "phaseA_ncc(8 dirs x views)", "view_select+final_costs", "current+refine(6 x sel views)"]
tot = sum(out[i] for i in range(5))
print(json.dumps({n: round(out[i] / tot, 4) for i, n in enumerate(names)}))
print(json.dumps({"candidates": out[5], "dup_of_earlier_candidate": out[6] / max(out[5], 1),
                  "equal_to_current_plane": out[7] / max(out[5], 1),
                  "unique_per_lane": out[11] / max(out[1 + 9] * 64, 1), "wave_max_unique": out[12] / max(out[10], 1),
                  "sel_views_per_lane": out[9] / max(out[10] * 64, 1), "sel_views_wave_union": out[8] / max(out[10], 1)}))
print(json.dumps({"ncc_lane_calls": out[16], "wave_box_le_512": out[13] / max(out[16], 1),
                  "wave_box_le_2048": out[14] / max(out[16], 1), "wave_box_le_8192": out[15] / max(out[16], 1)}))
