#!/bin/bash
# Round-4 A/B #5: geometric-cost depth fetches issued ahead (global loads,
# ACMMP_GEOM_AHEAD=7, the product) vs the same source with the fetches in
# place (ga0) vs the previous commit (head): per-pass launch times
# interleaved, the cfg2 bench, then the parity files that run geometric
# passes on the product build.
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
 "500 pt $V/libacmmp_amd_head.so $V/libacmmp_amd_ga0.so $B $V/libacmmp_amd_head.so $V/libacmmp_amd_ga0.so $B" \
 "400 bash tools/ab_bench.sh $V/libacmmp_amd_head.so $B $V/libacmmp_amd_head.so $B" \
 "600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_sweep_views.py tests/test_gpu_texel_modes.py tests/test_gpu_planar.py -x -q --timeout 200 --timeout-method thread"
