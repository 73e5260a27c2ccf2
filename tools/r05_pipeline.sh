#!/bin/bash
# Round 5: the 49-view cfg4 pipeline on one GPU with this round's library:
# the Python view-parallel driver, the C++ view-parallel driver (both world 1,
# Jacobi, 2 views in flight), the sequential CLI, and RunFusion of its maps.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "1000 python3 -u tools/pipeline_times.py 49 1600 1200 20 distributed,cli_vp,cli,fusion > gpurun_out/pipeline_r05.jsonl"
