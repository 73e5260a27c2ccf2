#!/bin/bash
# Round-4 A/B #4: pair records (dwordx2 gathers serving two samples) vs the
# product and the pair-load upper bound; parity of the pair build.
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "300 bash tools/pmc_ab.sh base=$B ubpair=$V/libacmmp_amd_ubpair.so pair=$V/libacmmp_amd_pair.so" \
 "100 python3 tools/pmc_ab.py gpurun_out/ab_base gpurun_out/ab_ubpair gpurun_out/ab_pair" \
 "400 bash tools/ab_bench.sh $B $V/libacmmp_amd_ubpair.so $V/libacmmp_amd_pair.so $B $V/libacmmp_amd_ubpair.so $V/libacmmp_amd_pair.so" \
 "400 ACMMP_LIB=$V/libacmmp_amd_pair.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_texel_modes.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread"
