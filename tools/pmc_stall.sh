#!/bin/bash
# Where k_sweep's waves spend their cycles: one PMC pass of SQ wave-state
# counters over tools/quick_time.py (3 photometric RunPatchMatch at cfg2),
# summarised per k_sweep launch by tools/pmc_phase.py.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d gpurun_out/pmc_stall -o run -- \
  python3 tools/quick_time.py 1600 1200 8 > gpurun_out/pmc_stall.log 2>&1 || exit $?
python3 tools/pmc_phase.py gpurun_out/pmc_stall
