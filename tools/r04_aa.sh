set -o pipefail
OUT=gpurun_out/${1:-r04aa}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u bench.py --config C4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('C4', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('C2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(r['frac'],3), r.get('isolated',{}).get('frac'))
print('header', d['latency']['header_digest_6667_parents']['p50_ms'], 'lone', d['digest']['single_chain']['ns_per_block'], 'c4share', d['digest']['c4_share']['kernel_ms'])
w=d['worker_digest']['windows']; print({k:(round(x['batches_per_s']), round(x['p50_latency_ms'],1)) for k,x in w.items()})"
exit 0
