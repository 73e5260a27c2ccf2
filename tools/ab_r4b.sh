#!/bin/bash
# Round-4 A/B #2: lane map 2 (+ easy patch, + h16 records) and the coherent-
# refinement upper bound (wrong results, timing only). Usage (GPU box).
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "500 bash tools/pmc_ab.sh base=$B m2=$V/libacmmp_amd_m2.so ubc=$V/libacmmp_amd_ubc.so ubcm2=$V/libacmmp_amd_ubcm2.so" \
 "120 python3 tools/pmc_ab.py gpurun_out/ab_base gpurun_out/ab_m2 gpurun_out/ab_ubc gpurun_out/ab_ubcm2" \
 "500 bash tools/ab_bench.sh $B $V/libacmmp_amd_m2.so $V/libacmmp_amd_m2e.so $V/libacmmp_amd_ubc.so $V/libacmmp_amd_ubcm2.so $B $V/libacmmp_amd_m2.so $V/libacmmp_amd_m2e.so" \
 "300 ACMMP_TEXEL=h16 bash tools/ab_bench.sh $B $V/libacmmp_amd_m2.so $V/libacmmp_amd_m2e.so"
