"""Interleaved wall times of acmmp_main binaries on the synthetic cfg4 folder
(tools/pipeline_times.write_cfg4_dense): each round runs every binary once,
in order, into its own output folder.

usage: python tools/cli_ab.py <rounds> <binary> [<binary> ...] > gpurun_out/cli_ab.jsonl
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
    from pipeline_times import write_cfg4_dense
    rounds, bins = int(sys.argv[1]), sys.argv[2:]
    tmp, dense = write_cfg4_dense(49, 1600, 1200, 20)
    for r in range(rounds):
        for k, b in enumerate(bins):
            out = "/ACMMP_ab%d" % k
            t0 = time.perf_counter()
            subprocess.run([b, dense, "--output_dir", out, "--no_fusion", "--quiet"], check=True)
            print(json.dumps({"round": r, "binary": os.path.basename(b), "s": round(time.perf_counter() - t0, 2)}),
                  flush=True)
            shutil.rmtree(dense + out, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
