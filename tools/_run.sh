set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
run() {  # tag, bench args
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 ${@:2} > gpurun_out/b_$1.log 2>&1 || { tail -5 gpurun_out/b_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/b_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; e=r['exact_kernel']; c=j.get('contrast_data'); print('$1', 'qps %.0f scan_ms %.3f exact_ms %.3f same %s merge %.3f plan %.3f bitexact %s recall %s tflops %.1f work %s' % (j['value'], j['kernels_ms_per_step']['scan'], e['scan_ms'], e['same_output_full_batch'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], j['parity_bit_exact'], j.get('recall_at_k'), r['compute']['achieved'], {a: round(b, 4) if isinstance(b, float) else b for a, b in r['work'].items()})); print('   contrast', c)"
}
run sift1m --config sift1m
run gist1m --config gist1m
run deep10m --config deep10m
run bigann100m --config bigann100m
