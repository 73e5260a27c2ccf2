#!/bin/bash
# Round-4 A/B of k_sweep lane maps and the easy-patch path: counters (3
# passes each), bench per library (u8 and h16 records), and the parity files
# against the most changed build. Usage (GPU box): bash tools/ab_r4.sh
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "500 bash tools/pmc_ab.sh base=$B m3=$V/libacmmp_amd_m3.so m3e=$V/libacmmp_amd_m3e.so e=$V/libacmmp_amd_e.so" \
 "120 python3 tools/pmc_ab.py gpurun_out/ab_base gpurun_out/ab_m3 gpurun_out/ab_m3e gpurun_out/ab_e" \
 "400 bash tools/ab_bench.sh $B $V/libacmmp_amd_m3.so $V/libacmmp_amd_m3e.so $V/libacmmp_amd_e.so $V/libacmmp_amd_m1.so $V/libacmmp_amd_m2.so" \
 "300 ACMMP_TEXEL=h16 bash tools/ab_bench.sh $B $V/libacmmp_amd_m3.so $V/libacmmp_amd_m3e.so" \
 "300 ACMMP_LIB=$V/libacmmp_amd_m3e.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread"
