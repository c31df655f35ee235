# Round-4 closing measurements (one GPU): tests, the default bench line, the rocprof cross-check of the
# headline's k_verify launches, per-config lines, C4.
set -o pipefail
OUT=gpurun_out/${1:-r04final}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(r['frac'],3), r.get('isolated',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kv -o kv -- python3 bench.py --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 > $OUT/bench_kv.json 2> $OUT/prof_kv.log || { echo "ROCPROF KV FAILED"; tail -20 $OUT/prof_kv.log; exit 1; }
python3 tools/roofline_rocprof.py $OUT/prof_kv/kv_kernel_trace.csv --bench $OUT/bench_kv.json --skip 2 --take 10 > $OUT/roofline_rocprof.json && cat $OUT/roofline_rocprof.json
timeout -k 10 500 python3 -u tools/bench_configs.py --only C1,C3,C5,W --cpu-seconds 3 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "CONFIGS FAILED"; tail -20 $OUT/configs.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); print(d['config'], round(d['sigs_per_s']/1e6,1), round(d['ms_per_step'] if 'ms_per_step' in d else d.get('ms_per_batch',0),3), d.get('parity'))"
timeout -k 10 400 python3 -u bench.py --config C4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('C4', round(d['value']/1e6,1), round(d['ms_per_step'],3), d['cpu_baseline']['value'])"
exit 0
