set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
run() {  # tag, bench args
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 ${@:2} > gpurun_out/b_$1.log 2>&1 || { tail -5 gpurun_out/b_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/b_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; print('$1', 'qps %.0f scan_ms %.3f noprune_ms %.3f merge %.3f exact %s recall %s valu %.1f work %s' % (j['value'], j['kernels_ms_per_step']['scan'], r['no_prune']['scan_ms'], j['kernels_ms_per_step']['merge'], j['parity_bit_exact'], j.get('recall_at_k'), r['valu']['achieved'], {a: round(b, 3) if isinstance(b, float) else b for a, b in r['work'].items()}))"
}
run sift1m --config sift1m
run sift1m_mix --config sift1m --data mixture
run gist1m --config gist1m
run deep10m --config deep10m
run bigann100m --config bigann100m
