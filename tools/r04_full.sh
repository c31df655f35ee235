# Round 4 GPU call: lone-chain clock probe, all GPU tests, host_fed repetitions, full default bench.
set -o pipefail
OUT=gpurun_out/${1:-r04g}; mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_PROBE" ]; then
timeout -k 10 180 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep x_mode $OUT/sha_lone.jsonl | cut -c1-330
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u tools/host_fed_reps.py 20 > $OUT/host_fed_reps.json 2> $OUT/host_fed_reps.err || { echo "HOSTFED FAILED"; tail -5 $OUT/host_fed_reps.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/host_fed_reps.json')); print('host_fed', d['median_ms'], [round(p['ms'],2) for p in d['passes']], d.get('cgroup_cpu_stat_delta'))"
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d.get('worker_digest'))[:1500]); print(json.dumps(d.get('host_fed'))[:400])"
exit 0
