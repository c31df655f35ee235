set -o pipefail
OUT=gpurun_out/${1:-r04v}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('C2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['frac'],3), d['roofline'].get('isolated',{}).get('frac'))
print('msm', round(d['msm']['value']/1e6,2), round(d['msm']['ms'],3))
print('host_fed', round(d['host_fed']['value']/1e6,1), [round(x,2) for x in d['host_fed']['ms_reps']], [round(x,2) for x in d['host_fed']['fresh_buffers']['ms_reps']])
w=d['worker_digest']['windows']; print('worker', {k:(round(v['batches_per_s']), round(v['p50_latency_ms'],1)) for k,v in w.items()})"
timeout -k 10 300 python3 -u tools/worker_probe.py > $OUT/worker_probe.jsonl 2> $OUT/worker_probe.err || { echo "PROBE FAILED"; tail -20 $OUT/worker_probe.err; exit 1; }
cat $OUT/worker_probe.jsonl | head -4
exit 0
