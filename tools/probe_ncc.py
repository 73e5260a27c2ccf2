"""Split-kernel NCC throughput probe (diagnostic; ACMMP_DIAG_PROBE build):
lean one-thread-per-(pixel, candidate) kernel, variants 0/1 = column-order
gathers (plain / pipelined), 2 = row-order gathers; on random (init-only)
and on converged (8-iteration) hypotheses.
usage: ACMMP_LIB=acmmp_amd/lib/variants/libacmmp_amd_probe.so python tools/probe_ncc.py"""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from acmmp_amd import ACMMP, default_params, scene, _abi

lib = _abi.load_library()
fn = lib.acmmp_diag_probe
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]
dev = torch.device("cuda", 0)
setup = scene.scene_setup(num_views=10, width=1600, height=1200)
ids = [0] + setup.pairs[0][:9]
imgs = [scene.render_torch(setup, i, dev) for i in ids]
for iters in (0, 8):
    eng = ACMMP(0)
    p = default_params()
    p.max_iterations = iters
    eng.set_params(p)
    eng.set_timing(True)
    eng.set_images_device([setup.camera(i) for i in ids], [im.data_ptr() for im in imgs])
    eng.RunPatchMatch()
    for variant in (0, 1, 2):
        ms = C.c_float(0)
        rc = fn(eng._ctx, variant, 5, C.byref(ms))
        print(f"state after {iters} iters: variant {variant} rc {rc} ms {ms.value:.3f} "
              f"per 960k-NCC-pass us {1000 * ms.value / 81:.1f}", flush=True)
    eng.close()
