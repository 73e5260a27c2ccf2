#!/bin/bash
# Round-4 wave-state counters before (r04pre: the kernel at 93c34e8) and
# after the latency fixes (the product): three rocprofv3 --pmc passes each.
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "400 bash tools/pmc_ab.sh pre=$V/libacmmp_amd_r04pre.so product=$B" \
 "100 python3 tools/pmc_ab.py gpurun_out/ab_pre gpurun_out/ab_product"
