set -o pipefail
OUT=gpurun_out/${1:-r04n}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u tools/worker_probe.py > $OUT/worker_probe.jsonl 2> $OUT/worker_probe.err || { echo "PROBE FAILED"; tail -20 $OUT/worker_probe.err; exit 1; }
cat $OUT/worker_probe.jsonl
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('C2', d['value']/1e6, d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['worker_digest'])[:700])"
timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('C4 default', d['value']/1e6, d['ms_per_step'])"
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_ldspad.so timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_ldspad.json 2> $OUT/bench_c4_ldspad.err || { echo "C4 LDSPAD FAILED"; tail -20 $OUT/bench_c4_ldspad.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4_ldspad.json').read().strip().splitlines()[-1]); print('C4 ldspad', d['value']/1e6, d['ms_per_step'])"
exit 0
