set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
one() {  # tag, env, args
    env $2 timeout -k 10 400 python -u bench.py --no-cpu-baseline --contrast none --steps 10 --recall-sample 20 ${@:3} > gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/ab_$1.log').read().strip().splitlines()[-1]); r=j['roofline']; e=r['exact_kernel']; print('$1', 'qps %.0f step %.3f scan_ms %.3f exact_ms %.3f same %s merge %.3f plan %.3f bitexact %s tflops %.1f surv %d' % (j['value'], j['ms_per_step'], j['kernels_ms_per_step']['scan'], e['scan_ms'], e['same_output_full_batch'], j['kernels_ms_per_step']['merge'], j['kernels_ms_per_step']['plan'], j['parity_bit_exact'], r['compute']['achieved'], r['work']['survivors']))"
}
one mix "X=0" --config sift1m
one mix_d8 "LIRA_SCAN_DEBUG=8" --config sift1m
grep work_raw gpurun_out/ab_mix_d8.log
one lat "X=0" --config sift1m --data latent
one gist "X=0" --config gist1m
one gist_lat "X=0" --config gist1m --data latent
one deep "X=0" --config deep10m
one big "X=0" --config bigann100m
