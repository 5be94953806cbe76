set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -x -v --timeout 120 --timeout-method thread -k "duplicate or fma or early or two_phase" > gpurun_out/t_scan.log 2>&1; rc=$?
tail -30 gpurun_out/t_scan.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
