#!/bin/bash
# Round-4 A/B #7: all 8 checkerboard searches load their 72 costs before
# any comparison and the reference tile loads are batched (the product) vs
# the previous product (prev, one batch per search): per-pass
# launch times interleaved, the cfg2 bench, then the parity files.
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
pt() {  # per-pass launch times of one library, appended to gpurun_out/pass_ab.jsonl
  for lib in "$@"; do
    echo -n "{\"lib\": \"$lib\", \"t\": " >> gpurun_out/pass_ab.jsonl
    ACMMP_LIB=$lib timeout -k 10 120 python3 tools/pass_times.py 2 >> gpurun_out/pass_ab.jsonl || return $?
    echo "}" >> gpurun_out/pass_ab.jsonl
  done
}
export -f pt
bash tools/gpu_steps.sh \
 "400 pt $V/libacmmp_amd_prev.so $B $V/libacmmp_amd_prev.so $B" \
 "400 bash tools/ab_bench.sh $V/libacmmp_amd_prev.so $B $V/libacmmp_amd_prev.so $B" \
 "600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sweep_views.py tests/test_gpu_texel_modes.py tests/test_gpu_planar.py tests/test_gpu_band.py -x -q --timeout 200 --timeout-method thread"
