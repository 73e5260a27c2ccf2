#!/bin/bash
# Round 5: Phase A alone (ACMMP_PHASE_A_ONLY, timing-only builds) so the
# shared-plane bounds do not change the downstream work: one call at a time
# (pa0), the pipelined stream (pa), and 2 / 8 / 64 lanes on one pixel's plane
# (pa2, pa8, pa64; wrong costs). Three PMC passes each (tools/pmc_ab.sh).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
timeout -k 10 900 bash tools/pmc_ab.sh pa0=$V/libacmmp_amd_pa0.so pa=$V/libacmmp_amd_pa.so pa2=$V/libacmmp_amd_pa2.so \
  pa8=$V/libacmmp_amd_pa8.so pa64=$V/libacmmp_amd_pa64.so && \
timeout 120 python3 tools/pmc_ab.py gpurun_out/ab_pa0 gpurun_out/ab_pa gpurun_out/ab_pa2 gpurun_out/ab_pa8 gpurun_out/ab_pa64 \
  > gpurun_out/phase_a_pmc.txt
rc=$?
grep -E "^== |per buffer|TD busy|wait_any|SQ_INSTS_VALU  " gpurun_out/phase_a_pmc.txt
rm -rf gpurun_out/ab_pa*
exit $rc
