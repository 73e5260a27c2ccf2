#!/bin/bash
# Round 5: timing-only upper bounds for lanes sharing one pixel's plane
# (ACMMP_UB_SHARE = 2, 8; wrong results) against the product (pipelined
# Phase A) and the pre-pipeline kernel: per-pass launch times and the three
# PMC passes of tools/pmc_ab.sh (SQ wave states, LDS/VMEM counts, TCP accesses).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "500 bash tools/ab.sh pass base=$V/libacmmp_amd_base.so pipe=$B ub2=$V/libacmmp_amd_ub2.so ub8=$V/libacmmp_amd_ub8.so" \
 "900 bash tools/ab.sh pmc base=$V/libacmmp_amd_base.so pipe=$B ub2=$V/libacmmp_amd_ub2.so ub8=$V/libacmmp_amd_ub8.so"
du -sh gpurun_out/* 2>/dev/null | sort -h | tail -5
