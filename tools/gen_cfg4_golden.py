"""Golden digests of cfg4's schedule at a reduced view size (TEST FIXTURE
GENERATOR; runs on the CPU oracle, about two hours on 6 threads).

cfg4 (BASELINE.json configs[3]) is 49 views with their 20 best sources each
(N = 21, colmap2mvsnet_acm.py:415), two scales with JBU + hierarchy + planar
prior and two geometric passes per scale (src/main_ACMMP.cpp:96-176). The
oracle pipeline over it takes hours even at reduced size, far beyond a GPU
test's budget, so this script runs it ONCE here and commits only digests:

  * the SHA-256 of every input file of the dense folder (22 views at
    1010x760, which ComputeMultiScaleSettings splits into 505x380 -> 1010x760,
    20 sources each), so the GPU test knows its inputs are these;
  * the SHA-256 of every output map (view, name) of
    OraclePipeline.run_multi_scale("jacobi"), over the float32 bytes with
    every NaN replaced by 0x7fc00000 (NaN payloads carry no meaning; the bit
    comparison of tests/parity_util.py treats any NaN as equal).

tests/test_gpu_cfg4.py rebuilds the same folder, runs both view-parallel
drivers at world 2 and compares digests.

Usage: OMP_NUM_THREADS=6 python tools/gen_cfg4_golden.py [out.json]
"""
import hashlib
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

NUM_VIEWS, WIDTH, HEIGHT, NUM_SRC = 22, 1010, 760, 20
OUT = os.path.join(ROOT, "tests", "golden", "cfg4_ms_n21.json")


def map_digest(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    u = a.view(np.uint32).copy()
    u[np.isnan(a)] = 0x7FC00000
    h = hashlib.sha256()
    h.update(np.asarray(a.shape, np.int64).tobytes())
    h.update(u.astype("<u4").tobytes())
    return h.hexdigest()


def file_digests(dense):
    out = {}
    for sub in ("images", "cams"):
        for name in sorted(os.listdir(os.path.join(dense, sub))):
            with open(os.path.join(dense, sub, name), "rb") as f:
                out[f"{sub}/{name}"] = hashlib.sha256(f.read()).hexdigest()
    with open(os.path.join(dense, "pair.txt"), "rb") as f:
        out["pair.txt"] = hashlib.sha256(f.read()).hexdigest()
    return out


def make_dense(folder):
    from acmmp_amd import scene
    sc = scene.make_scene(num_views=NUM_VIEWS, width=WIDTH, height=HEIGHT)
    scene.write_dense_folder(sc, folder, num_src=NUM_SRC)
    return sc


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else OUT
    from oracle_pipeline import OraclePipeline
    with tempfile.TemporaryDirectory() as d:
        make_dense(d)
        inputs = file_digests(d)
        t0 = time.time()
        maps = OraclePipeline(d).run_multi_scale("jacobi")
        dt = time.time() - t0
    res = {
        "what": "OraclePipeline.run_multi_scale('jacobi') of scene.make_scene(22, 1010, 760), 20 sources",
        "generator": "tools/gen_cfg4_golden.py",
        "oracle_seconds": round(dt, 1),
        "omp_threads": os.environ.get("OMP_NUM_THREADS"),
        "inputs": inputs,
        "maps": {f"{v}/{name}": map_digest(a) for (v, name), a in sorted(maps.items())},
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(f"{len(res['maps'])} map digests in {dt:.0f} s -> {out}")


if __name__ == "__main__":
    main()
