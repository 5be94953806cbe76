set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for cfg in sift1m gist1m bigann100m; do
    timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 10 > gpurun_out/b_${cfg}.log 2>&1 || { tail -5 gpurun_out/b_${cfg}.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/b_${cfg}.log').read().strip().splitlines()[-1]); r=j['roofline']; print('$cfg', 'qps %.0f scan_ms %.3f merge %.3f exact %s recall %s valu %.1f work %s' % (j['value'], j['kernels_ms_per_step']['scan'], j['kernels_ms_per_step']['merge'], j['parity_bit_exact'], j.get('recall_at_k'), r['valu']['achieved'], r['work']))"
done
