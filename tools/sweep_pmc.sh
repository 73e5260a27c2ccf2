#!/bin/bash
# k_sweep hardware counters of one source-count bucket, photometric and
# geometric launches side by side (replaces geom_pmc.sh, which did cfg2 only).
#
#   bash tools/sweep_pmc.sh <nsrc> [lib.so]     (nsrc 9 = cfg2, 20 = cfg4's fine scale)
#
# Five rocprofv3 --pmc passes of tools/pass_times.py 1 (nsrc + 1 views at
# 1600x1200, 8 iterations: a photometric then a geometric pass, twice), each
# within the gfx950 slot limits (SQ 8, TCC 4, TCP 4, TA 2, TD 2, GRBM 2);
# tools/sweep_pmc.py splits the last repetition's k_sweep dispatches into its
# photometric and geometric launches and prints per-launch means and the
# derived figures (TD busy, TCP accesses per gather, VALU share, scratch and
# state accesses against the gathers, write amplification) as text and JSON.
set -o pipefail
export TMPDIR=/tmp
ns=${1:?usage: tools/sweep_pmc.sh <nsrc> [lib.so]}
lib=${2:-acmmp_amd/lib/libacmmp_amd.so}
out=gpurun_out/sweep_pmc_ns$ns
rm -rf "$out"; mkdir -p "$out"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE TD_TD_BUSY_sum TA_TA_BUSY_sum"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SALU SQ_WAVES TA_BUFFER_READ_WAVEFRONTS_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum TA_BUFFER_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
P4="FETCH_SIZE TD_TD_BUSY_sum TD_STORE_WAVEFRONT_sum GRBM_GUI_ACTIVE"
P5="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for set in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  env ACMMP_LIB=$lib PASS_NSRC=$ns timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex k_sweep \
    --pmc $set -f csv -d "$out/p$i" -o run -- python3 tools/pass_times.py 1 > "$out/p$i.log" 2>&1
  rc=$?
  echo "nsrc $ns pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python3 tools/sweep_pmc.py "$out" "$ns" > "$out/summary.txt"
rc=$?; cat "$out/summary.txt"
# keep the summaries, drop the per-dispatch CSVs (tens of MB)
rm -rf "$out"/p[0-9]
exit $rc
