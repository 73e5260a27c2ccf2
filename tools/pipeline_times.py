"""End-to-end timing of the pass driver on BASELINE cfg4's shape on ONE GPU.

cfg4 (BASELINE.json configs[3]): 49 views at 1600x1200, each with its 20 best
source views (N = 21, colmap2mvsnet_acm.py:415), main_ACMMP's multi-scale loop
(src/main_ACMMP.cpp:96-176: planar-prior pass, geometric passes, JBU +
hierarchy on the finer scale). The reference runs it on 8 GPUs; here the
same folder runs on one GPU through

  distributed   acmmp_amd.distributed.ViewParallelPipeline (world 1, Jacobi
                order, 2 views in flight on 2 HIP streams)
  cli           acmmp_amd/lib/acmmp_main --no_fusion (the C++ driver,
                sequential Gauss-Seidel order, one engine)
  fusion        RunFusion over the CLI's maps (C++, host)

Synthetic, seeded scene rendered on the GPU and written as 8-bit JPEGs (a
COLMAP-converted dense folder); wall times include JPEG decode and .dmb I/O,
as the reference's do. Iterations: the driver's default (the reference's).
usage: python tools/pipeline_times.py [views] [width] [height] [nsrc] [steps] > gpurun_out/pipeline.jsonl
  steps: comma list of distributed,cli_vp,cli,cli_serial,fusion,fusion_dist (default distributed,cli,fusion;
         cli_serial also runs the CLI with --concurrent_views 1 and compares the two's maps;
         fusion fuses the CLI's maps, fusion_dist the distributed driver's, once per library in
         ACMMP_FUSION_LIBS (comma list, default the product) in a subprocess each)

The 49 views sit 1.8 degrees apart on the arc (86 degrees in all, like a DTU
scan; r01/r02 used 6 degrees, which wraps 288 degrees round the object and
leaves some views looking at the scene edge-on).
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acmmp_amd import scene  # noqa: E402
from acmmp_amd import pipeline  # noqa: E402
from acmmp_amd.distributed import ViewParallelPipeline  # noqa: E402
from acmmp_amd import load_library as _lib  # noqa: E402

_argv = sys.argv if __name__ == "__main__" else []
V = int(_argv[1]) if len(_argv) > 1 else 49
W = int(_argv[2]) if len(_argv) > 2 else 1600
H = int(_argv[3]) if len(_argv) > 3 else 1200
NSRC = int(_argv[4]) if len(_argv) > 4 else 20
STEPS = set((_argv[5] if len(_argv) > 5 else "distributed,cli,fusion").split(","))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def cgroup_cpu_stat() -> dict:
    """cgroup v2 cpu.stat counters (usage / throttling), {} if unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if line.strip())}
    except (OSError, ValueError):
        return {}


def write_cfg4_dense(V, W, H, NSRC):
    """The synthetic cfg4-shaped dense folder (rendered on cuda:0); returns (tmp, dense)."""
    dev = torch.device("cuda", 0)
    setup = scene.scene_setup(num_views=V, width=W, height=H, arc_deg=float(os.environ.get("ACMMP_ARC_DEG", "1.8")))
    views = []
    for i in range(V):
        img = scene.render_torch(setup, i, dev).cpu().numpy()
        R, t, _, _ = setup.poses[i]
        views.append(scene.View(K=setup.K.astype(np.float32), R=R.astype(np.float32), t=t.astype(np.float32),
                                image=img, depth=None, normal=None))
    sc = scene.Scene(views=views, pairs=setup.pairs)
    tmp = tempfile.mkdtemp(prefix="acmmp_cfg4_")
    dense = os.path.join(tmp, "dense")
    scene.write_dense_folder(sc, dense, num_src=NSRC)
    return tmp, dense


def main():
    t0 = time.perf_counter()
    tmp, dense = write_cfg4_dense(V, W, H, NSRC)
    emit(step="write_dense", views=V, width=W, height=H, nsrc=NSRC, s=round(time.perf_counter() - t0, 2))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            cpu_max = f.read().strip()
    except OSError:
        cpu_max = None
    emit(step="host", cgroup_cpu_max=cpu_max, affinity_cpus=len(os.sched_getaffinity(0)),
         host_threads=int(_lib().acmmp_host_threads()))

    if "distributed" in STEPS:
        t0 = time.perf_counter()
        pipe = ViewParallelPipeline(dense, "/ACMMP_dist", device=0, concurrent_views=2, timing=True)
        pipe.run()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        # gpu_runpatchmatch_s: the runs' HIP-event durations summed (two views
        # overlap on the GPU, so the sum can exceed the compute phase's wall)
        emit(step="distributed_world1", order="jacobi", concurrent_views=2, s=round(wall, 2),
             gpu_runpatchmatch_s=round(pipe.gpu_ms / 1e3, 2),
             phases_s={k: round(v, 2) for k, v in sorted(pipe.phase_s.items())})
        if "fusion_dist" in STEPS:
            # per library (ACMMP_FUSION_LIBS) and host-thread count
            # (ACMMP_FUSION_THREADS, default the library's own budget), one
            # subprocess each; the cgroup's CPU throttling over the call is
            # reported beside the time
            threads = [t for t in os.environ.get("ACMMP_FUSION_THREADS", "").split(",") if t]
            for lib in os.environ.get("ACMMP_FUSION_LIBS", os.path.join(ROOT, "acmmp_amd", "lib",
                                                                         "libacmmp_amd.so")).split(","):
                for nt in threads or [None]:
                    code = ("import sys, time, json; sys.path.insert(0, %r); from acmmp_amd import pipeline; "
                            "t0 = time.perf_counter(); n = pipeline.run_fusion(%r, %r); "
                            "print(json.dumps({'points': n, 's': round(time.perf_counter() - t0, 2)}))"
                            % (ROOT, dense, dense + "/ACMMP_dist"))
                    env = dict(os.environ, ACMMP_LIB=lib)
                    if nt:
                        env["ACMMP_HOST_THREADS"] = nt
                    c0 = cgroup_cpu_stat()
                    r = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True, check=True,
                                       env=env)  # stderr: ACMMP_HOST_TIMING lines
                    c1 = cgroup_cpu_stat()
                    res = json.loads(r.stdout.strip().splitlines()[-1])
                    emit(step="fusion_of_distributed_maps", lib=os.path.basename(lib), points=res["points"],
                         s=res["s"], host_threads=int(nt) if nt else int(_lib().acmmp_host_threads()),
                         cgroup_delta={k: c1[k] - c0.get(k, 0) for k in c1})
        shutil.rmtree(dense + "/ACMMP_dist", ignore_errors=True)
    if "cli_vp" in STEPS:  # the C++ view-parallel driver, world 1 (no communicator: a device copy stands for the all-gather)
        cli = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT="29611")
        t0 = time.perf_counter()
        subprocess.run([cli, dense, "--view_parallel", "--output_dir", "/ACMMP_cvp", "--no_fusion", "--quiet"],
                       stdout=sys.stderr, check=True, env=env)
        emit(step="cli_view_parallel_world1", order="jacobi", concurrent_views=2, exchange="device copy (world 1 default)",
             s=round(time.perf_counter() - t0, 2))
        shutil.rmtree(dense + "/ACMMP_cvp", ignore_errors=True)
    if "cli" not in STEPS:
        shutil.rmtree(tmp, ignore_errors=True)
        return

    cli = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")

    def cli_serial():  # one view at a time in every pass (--concurrent_views 1)
        t0 = time.perf_counter()
        subprocess.run([cli, dense, "--output_dir", "/ACMMP_serial", "--no_fusion", "--concurrent_views", "1"],
                       stdout=sys.stderr, check=True)
        emit(step="cli_serial", order="sequential", concurrent_views=1, s=round(time.perf_counter() - t0, 2))

    # cli_serial runs before the default CLI; cli_serial_last after it (the
    # first run of a call meets colder file caches)
    if "cli_serial" in STEPS and "cli_serial_last" not in STEPS:
        cli_serial()
    t0 = time.perf_counter()
    subprocess.run([cli, dense, "--output_dir", "/ACMMP", "--no_fusion"], stdout=sys.stderr, check=True)
    emit(step="cli", order="sequential", concurrent_views=2, s=round(time.perf_counter() - t0, 2))
    if "cli_serial_last" in STEPS:
        cli_serial()
    if "cli_serial" in STEPS:  # the non-geometric passes' views in flight change no output byte
        diff = [f for f in sorted(os.listdir(dense + "/ACMMP_serial")) for m in ("depths_geom.dmb", "normals.dmb",
                                                                                   "costs.dmb")
                if open(os.path.join(dense, "ACMMP_serial", f, m), "rb").read()
                != open(os.path.join(dense, "ACMMP", f, m), "rb").read()]
        emit(step="cli_vs_cli_serial", identical=not diff, differing=diff[:5])
        shutil.rmtree(dense + "/ACMMP_serial", ignore_errors=True)

    t0 = time.perf_counter()
    n = pipeline.run_fusion(dense, dense + "/ACMMP")
    emit(step="fusion", points=n, s=round(time.perf_counter() - t0, 2))
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
