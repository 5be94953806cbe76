set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
one() {  # tag, env, args
    env $2 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --recall-sample 20 ${@:3} > gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; e=r['exact_kernel']; print('$1', 'qps %.0f scan_ms %.3f exact_ms %.3f same %s merge %.3f plan %.3f bitexact %s valu %.1f surv %d rechk %d' % (j['value'], j['kernels_ms_per_step']['scan'], e['scan_ms'], e['same_output_full_batch'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], j['parity_bit_exact'], r['compute']['achieved'], r['work']['survivors'], r['work']['rechecked']))"
}
for cfg in sift1m gist1m deep10m bigann100m; do
  one ${cfg}_mfma X=1 --config $cfg
  one ${cfg}_valu LIRA_SCAN_MFMA=0 --config $cfg
done
