#!/bin/bash
# Round 5: RunFusion on cfg4 maps, 7 interleaved rounds: the approval walk
# without prefetch (nopf = make variant NAME=nopf EXTRA=-DACMMP_WALK_PREFETCH=0),
# prefetching the source-mask words 16 / 48 (product) / 128 hits ahead
# (pf16, pf128 = make variant NAME=pfN EXTRA=-DACMMP_WALK_PREFETCH=N).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
bash tools/gpu_steps.sh \
 "800 python3 tools/fusion_ab.py '[{\"ACMMP_LIB\": \"$V/libacmmp_amd_nopf.so\"}, {\"ACMMP_LIB\": \"$V/libacmmp_amd_pf16.so\"}, {}, {\"ACMMP_LIB\": \"$V/libacmmp_amd_pf128.so\"}]' 7 > gpurun_out/walk_prefetch_ab.jsonl"
