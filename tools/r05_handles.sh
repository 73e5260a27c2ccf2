#!/bin/bash
# Round 5: engine streams and events cached with the device blocks: the whole
# GPU suite, then the cfg4 sequential CLI with the caches on (default) and
# off (ACMMP_DEVICE_POOL_MB=0), 3 interleaved rounds.
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
 "1000 python -u -m pytest tests -x -m gpu -q --durations=10 --timeout 300 --timeout-method thread" \
 "700 python3 -u tools/cli_ab.py 3 acmmp_amd/lib/acmmp_main ACMMP_DEVICE_POOL_MB=0@acmmp_amd/lib/acmmp_main > gpurun_out/cli_handles.jsonl"
