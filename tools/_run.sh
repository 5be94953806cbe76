set -o pipefail
mkdir -p gpurun_out
run() {  # tag, bench args
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 ${@:2} > gpurun_out/b_$1.log 2>&1 || { tail -5 gpurun_out/b_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/b_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; e=r['exact_kernel']; print('$1', 'qps %.0f scan_ms %.3f exact_ms %.3f same %s merge %.3f plan %.3f rank %.3f bitexact %s recall %s valu %.1f work %s' % (j['value'], j['kernels_ms_per_step']['scan'], e['scan_ms'], e['same_output_full_batch'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], j['kernels_ms_per_step']['rank_nearest'], j['parity_bit_exact'], j.get('recall_at_k'), r['valu']['achieved'], {a: round(b, 4) if isinstance(b, float) else b for a, b in r['work'].items()}))"
}
run sift1m --config sift1m
run gist1m --config gist1m
#run deep10m --config deep10m
#run bigann100m --config bigann100m
#run sift1m_mix --config sift1m --data mixture
