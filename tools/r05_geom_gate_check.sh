#!/bin/bash
# Round 5: after gating the geometric fetch-ahead to the 9-view bucket, the
# hot-path parity files on the product, then per-pass times at nsrc 21 (NS 32)
# against the bit-0-off variant (they should now match).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
rm -f gpurun_out/ab_pass.jsonl
bash tools/ab.sh parity prod=acmmp_amd/lib/libacmmp_amd.so || exit $?
PASS_NSRC=21 bash tools/ab.sh pass prod=acmmp_amd/lib/libacmmp_amd.so ga6=$V/libacmmp_amd_ga6.so || exit $?
