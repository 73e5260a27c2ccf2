"""cfg4's real shape (BASELINE configs[3]: 49 views at 1600x1200, 20 sources
each, main_ACMMP's multi-scale schedule) through the C++ view-parallel driver
at world 1 and at world 8 on ONE GPU (8 ranks sharing the device through the
TCP exchange: RCCL refuses several ranks on one device), tail views split in
row bands over the ranks. Every .dmb of the two runs must be byte-identical.
usage (GPU box): python tools/cfg4_world8_rehearsal.py [views] [world] > gpurun_out/cfg4_w8.json"""
import filecmp
import json
import os
import shutil
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
EXE = os.path.join(ROOT, "acmmp_amd", "lib", "acmmp_main")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(dense, out, world, exchange, timeout=900):
    port = free_port()
    procs = []
    t0 = time.time()
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port - 1), ACMMP_RDZV_PORT=str(port))
        cmd = [EXE, dense, "--view_parallel", "--exchange", exchange, "--device", "0", "--output_dir", out,
               "--no_fusion", "--quiet"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    errs = []
    for p in procs:
        so, se = p.communicate(timeout=timeout)
        if p.returncode:
            errs.append((p.returncode, se[-2000:]))
    wall = time.time() - t0
    if errs:
        raise SystemExit("world %d failed: %s" % (world, errs[0]))
    return wall


def heartbeat():
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(30)
            print("... %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    from pipeline_times import write_cfg4_dense
    heartbeat()
    V = int(sys.argv[1]) if len(sys.argv) > 1 else 49
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    tmp, dense = write_cfg4_dense(V, 1600, 1200, 20)
    try:
        w1 = launch(dense, "/W1", 1, "tcp")
        print("world 1 done %.1f s" % w1, file=sys.stderr, flush=True)
        wn = launch(dense, "/WN", world, "tcp")
        print("world %d done %.1f s" % (world, wn), file=sys.stderr, flush=True)
        files = same = 0
        diff = []
        for dp, _, fs in os.walk(dense + "/W1"):
            for f in fs:
                if not f.endswith(".dmb"):
                    continue
                a = os.path.join(dp, f)
                b = a.replace(dense + "/W1", dense + "/WN", 1)
                files += 1
                if os.path.exists(b) and filecmp.cmp(a, b, shallow=False):
                    same += 1
                else:
                    diff.append(os.path.relpath(a, dense))
        print(json.dumps({"workload": "cfg4: %d views 1600x1200, 20 sources, multi-scale (C++ view-parallel driver)" % V,
                          "world_1_wall_s": round(w1, 2), "world_%d_wall_s" % world: round(wn, 2),
                          "world_note": "all ranks share ONE MI355X (TCP exchange); wall times include JPEG decode "
                                        "and .dmb I/O; tail views split in row bands over the ranks",
                          "dmb_files": files, "identical": same, "differing": diff[:10]}))
        if same != files or files == 0:
            sys.exit(1)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
