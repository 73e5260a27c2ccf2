"""Interleaved wall times of acmmp_main binaries on the synthetic cfg4 folder
(tools/pipeline_times.write_cfg4_dense): each round runs every binary once,
in order, into its own output folder.

usage: python tools/cli_ab.py <rounds> <side> [<side> ...] > gpurun_out/cli_ab.jsonl
  side: <binary> or VAR=value@<binary> (one environment variable for that side)
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
        for k, side in enumerate(bins):
            env = dict(os.environ)
            b = side
            if "@" in side:
                var, b = side.split("@", 1)
                env[var.split("=", 1)[0]] = var.split("=", 1)[1]
            out = "/ACMMP_ab%d" % k
            t0 = time.perf_counter()
            subprocess.run([b, dense, "--output_dir", out, "--no_fusion", "--quiet"], check=True, env=env)
            print(json.dumps({"round": r, "side": side, "s": round(time.perf_counter() - t0, 2)}), flush=True)
            shutil.rmtree(dense + out, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
