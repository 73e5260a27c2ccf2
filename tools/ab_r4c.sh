#!/bin/bash
# Round-4 A/B #3: block shape with lane map 2 (32x8, 8x32 vs 16x16), bench.
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "500 bash tools/ab_bench.sh $B $V/libacmmp_amd_bx32.so $V/libacmmp_amd_bx8.so $B $V/libacmmp_amd_bx32.so $V/libacmmp_amd_bx8.so"
