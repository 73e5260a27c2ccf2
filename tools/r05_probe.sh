export TMPDIR=/tmp
V=acmmp_amd/lib/variants
timeout -k 10 300 bash tools/pmc_ab.sh ub64=$V/libacmmp_amd_ub64.so && timeout 60 python3 tools/pmc_ab.py gpurun_out/ab_ub64 | grep -E "ms/launch|per buffer|TD busy|wait_any"
