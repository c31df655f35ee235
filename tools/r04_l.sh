set -o pipefail
OUT=gpurun_out/${1:-r04l}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python3 -u tools/bench_configs.py --only C3,C5 --cpu-seconds 0 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "CONFIGS FAILED"; tail -20 $OUT/configs.err; exit 1; }
cut -c1-300 $OUT/configs.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg -o cfg -- python3 tools/bench_configs.py --only C5 --cpu-seconds 0 --steps 3 > $OUT/prof_cfg.log 2>&1 || { echo "PROF CONFIG FAILED"; tail -20 $OUT/prof_cfg.log; exit 1; }
f=$(find $OUT/prof_cfg -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_c5.csv && cut -d, -f1-4 $OUT/kernel_stats_c5.csv | cut -c1-150 | head -16
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac'])
print('latency', {k: round(v['p50_ms'],4) for k, v in d['latency'].items() if isinstance(v, dict)})
print('worker', {k: (round(v['batches_per_s']), round(v['p50_latency_ms'],1)) for k, v in d['worker_digest']['windows'].items()})
print('host_fed', [round(x,2) for x in d['host_fed']['ms_reps']], [round(x,2) for x in d['host_fed']['fresh_buffers']['ms_reps']])
print('msm', d['msm']['value']/1e6)
"
timeout -k 10 300 python3 -u tools/worker_probe.py > $OUT/worker_probe.jsonl 2> $OUT/worker_probe.err || { echo "WORKER PROBE FAILED"; tail -5 $OUT/worker_probe.err; exit 1; }
cat $OUT/worker_probe.jsonl
exit 0
