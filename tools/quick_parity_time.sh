set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/quick_time.py 1600 1200 8 > gpurun_out/ts_time.log 2>&1 || exit $?
grep -o '"launch_ms": [0-9.]*' gpurun_out/ts_time.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep_views.py tests/test_gpu_headline.py tests/test_gpu_texel_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ts_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/ts_tests.log; exit $rc
