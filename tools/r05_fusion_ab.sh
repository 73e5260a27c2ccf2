#!/bin/bash
# Round 5: RunFusion on cfg4 maps, 7 interleaved rounds: round-start library
# (base = make variant NAME=base REV=c228eaf), world points from phase 1
# (fwp = make variant NAME=fwp REV=<the build compared>), and the product (walk over the
# phase-1 live pixels only).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
bash tools/gpu_steps.sh \
 "700 python3 tools/fusion_ab.py '[{\"ACMMP_LIB\": \"$V/libacmmp_amd_fwp.so\"}, {}]' 11 > gpurun_out/fusion_ab5.jsonl"
