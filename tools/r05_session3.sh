#!/bin/bash
# Round 5, GPU session 2b: per-pass A/B of the geometric wave-uniform view
# skip (product) against the round-start kernel (base); the default bench line (with the L2 counter pass),
# torchrun rehearsals of the N>1 bench line, the fusion walk A/B (7
# interleaved rounds, round-4 library vs the product).
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
B=acmmp_amd/lib/libacmmp_amd.so
bash tools/gpu_steps.sh \
 "300 bash tools/ab.sh pass base=$V/libacmmp_amd_base.so wv=$B" \
 "700 python3 bench.py > gpurun_out/bench.log 2>&1; grep ^{ gpurun_out/bench.log | tail -n 1 > gpurun_out/bench.json" \
 "400 bash tools/rehearse_bench.sh" \
 "500 python3 tools/fusion_ab.py '[{\"ACMMP_LIB\": \"$V/libacmmp_amd_base.so\"}, {}]' 7 > gpurun_out/fusion_ab.jsonl"
rm -rf gpurun_out/bench_pmc
du -sh gpurun_out/* 2>/dev/null | sort -h | tail -4
