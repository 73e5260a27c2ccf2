#!/bin/bash
# Round 5: the pipelined Phase A (product) against the previous kernel
# (variants/base = make variant NAME=base REV=<pre-pipeline commit>): hot-path
# parity of the product, per-pass launch times and bench, interleaved.
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sweep_views.py -m gpu -x -q --timeout 200 --timeout-method thread" \
 "500 bash tools/ab.sh pass base=$V/libacmmp_amd_base.so pipe=$B" \
 "500 bash tools/ab.sh bench base=$V/libacmmp_amd_base.so pipe=$B"
du -sh gpurun_out/* 2>/dev/null | sort -h | tail -5
