#!/bin/bash
# Round 5: the geometric final costs' fetch-ahead (ACMMP_GEOM_AHEAD
# bit 0) with more than 9 sources: per-pass launch times at nsrc 9 (NS 9
# kernels) and 16 (NS 16), product vs the same tree with bit 0 off
# (make -C acmmp_amd/csrc variant NAME=ga6 EXTRA="-DACMMP_GEOM_AHEAD=6").
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
rm -f gpurun_out/ab_pass.jsonl
PASS_NSRC=9 bash tools/ab.sh pass prod=acmmp_amd/lib/libacmmp_amd.so ga6=$V/libacmmp_amd_ga6.so || exit $?
PASS_NSRC=16 bash tools/ab.sh pass prod=acmmp_amd/lib/libacmmp_amd.so ga6=$V/libacmmp_amd_ga6.so || exit $?
