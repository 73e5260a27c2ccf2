#!/bin/bash
# Round 5: 512-thread blocks (a CU's 8 waves on adjacent pixels: 16 x 32 or
# 32 x 16 colour-split pixels) against the 256-thread product:
# make variant NAME=b512 EXTRA=-DACMMP_BLOCK_THREADS=512 (and ACMMP_KBX=32 for b512w).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "400 bash tools/ab.sh pass b256=$B b512=$V/libacmmp_amd_b512.so b512w=$V/libacmmp_amd_b512w.so" \
 "600 bash tools/ab.sh pmc b256=$B b512=$V/libacmmp_amd_b512.so b512w=$V/libacmmp_amd_b512w.so"
rm -rf gpurun_out/ab_b256 gpurun_out/ab_b512 gpurun_out/ab_b512w
