set -o pipefail
mkdir -p gpurun_out
one() {  # tag, env, args
    env $2 timeout -k 10 400 python -u bench.py --no-cpu-baseline --contrast none --steps 10 --recall-sample 4 ${@:3} > gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; e=r['exact_kernel']; print('$1', 'qps %.0f scan_ms %.3f exact_ms %.3f merge %.3f plan %.3f bitexact %s tflops %.1f surv %d' % (j['value'], j['kernels_ms_per_step']['scan'], e['scan_ms'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], j['parity_bit_exact'], r['compute']['achieved'], r['work']['survivors']))"
}
for dbg in 0 1 2 3; do one lat_dbg$dbg LIRA_SCAN_DEBUG=$dbg --config sift1m --data latent; done
one gist_lat X=0 --config gist1m --data latent
one gist_lat_dbg1 LIRA_SCAN_DEBUG=1 --config gist1m --data latent
one deep X=0 --config deep10m
