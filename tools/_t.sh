set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
