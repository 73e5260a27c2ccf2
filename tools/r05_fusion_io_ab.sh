#!/bin/bash
# Round 5: RunFusion on cfg4 maps, 7 interleaved rounds: the last commit
# (prev = make variant NAME=prev REV=<that commit>), one JPEG decode per
# view + the chunked parallel PLY write (mid = make variant NAME=mid), and
# the product (mid + the 9-bit AC lookahead table).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
bash tools/gpu_steps.sh \
 "700 python3 tools/fusion_ab.py '[{\"ACMMP_LIB\": \"$V/libacmmp_amd_prev.so\"}, {\"ACMMP_LIB\": \"$V/libacmmp_amd_mid.so\"}, {}]' 7 > gpurun_out/fusion_io_ab.jsonl"
