#!/bin/bash
# Round 5 closing evidence (1/2): the whole GPU suite as the driver runs it
# (-x), with the 30 slowest tests reported.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "1150 python -u -m pytest tests -x -m gpu -q --durations=30 --timeout 300 --timeout-method thread"
