set -o pipefail
mkdir -p gpurun_out
one() {  # tag, env, args
    env $2 timeout -k 10 400 python -u bench.py --no-cpu-baseline --contrast none --steps 10 --recall-sample 20 ${@:3} > gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; print('$1', 'qps %.0f step %.3f scan_ms %.3f merge %.3f plan %.3f tflops %.1f work %s' % (j['value'], j['ms_per_step'], j['kernels_ms_per_step']['scan'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], r['compute']['achieved'], r['work']))"
}
one mix X=0 --config sift1m
one mix_d1 LIRA_SCAN_DEBUG=1 --config sift1m
one mix_d2 LIRA_SCAN_DEBUG=2 --config sift1m
one mix_d3 LIRA_SCAN_DEBUG=3 --config sift1m
one mix_r4 LIRA_SCAN_ROUNDS=4 --config sift1m
one mix_r2 LIRA_SCAN_ROUNDS=2 --config sift1m
