#!/bin/bash
# Round 5: per-launch-index k_sweep durations (iterations 0..7, two colours)
# of the pre-pipeline kernel (base) and the pipelined product.
export TMPDIR=/tmp
V=acmmp_amd/lib/variants
for spec in base=$V/libacmmp_amd_base.so pipe=acmmp_amd/lib/libacmmp_amd.so base2=$V/libacmmp_amd_base.so pipe2=acmmp_amd/lib/libacmmp_amd.so; do
  n=${spec%%=*}; lib=${spec#*=}
  ACMMP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/lp_$n -o run -- python3 tools/quick_time.py 1600 1200 8 \
    > gpurun_out/lp_$n.log 2>&1 || exit $?
done
python3 tools/launch_profile.py gpurun_out/lp_base gpurun_out/lp_pipe gpurun_out/lp_base2 gpurun_out/lp_pipe2 | tee gpurun_out/launch_profile.jsonl
rm -rf gpurun_out/lp_*/
