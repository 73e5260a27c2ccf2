"""RunFusion A/B on cfg4-shaped maps: the synthetic cfg4 folder
(pipeline_times.write_cfg4_dense) through the distributed driver once, then
RunFusion in a subprocess per configuration, configurations interleaved
`repeat` times (the host is shared: interleaving spreads its noise).

usage: python tools/fusion_ab.py '<json list of env dicts>' [repeat] [views] [width] [height] [nsrc]
  e.g. '[{}, {"ACMMP_HOST_THREADS": "8"}]'
Prints one JSON line per run with RunFusion's own phase timing line.
"""
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    from acmmp_amd.distributed import ViewParallelPipeline
    from pipeline_times import write_cfg4_dense
    a = sys.argv
    configs = json.loads(a[1]) if len(a) > 1 else [{}]
    repeat = int(a[2]) if len(a) > 2 else 3
    V, W, H, NSRC = (int(a[k]) if len(a) > k else d for k, d in zip(range(3, 7), (49, 1600, 1200, 20)))
    tmp, dense = write_cfg4_dense(V, W, H, NSRC)
    ViewParallelPipeline(dense, "/ACMMP_fab", device=0).run()
    torch.cuda.synchronize()
    code = ("import sys, time, json; sys.path.insert(0, %r); from acmmp_amd import pipeline; "
            "t0 = time.perf_counter(); n = pipeline.run_fusion(%r, %r); "
            "print(json.dumps({'points': n, 's': round(time.perf_counter() - t0, 3)}))"
            % (ROOT, dense, dense + "/ACMMP_fab"))
    for r in range(repeat):
        for k, cfg in enumerate(configs):
            env = dict(os.environ, ACMMP_HOST_TIMING="1", **cfg)
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env)
            if p.returncode:
                print(p.stderr[-2000:], file=sys.stderr)
                raise SystemExit(p.returncode)
            res = json.loads(p.stdout.strip().splitlines()[-1])
            timing = [l for l in p.stderr.splitlines() if l.startswith("[RunFusion]")]
            print(json.dumps({"round": r, "config": k, "env": cfg, **res, "timing": timing[-1] if timing else None}),
                  flush=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
