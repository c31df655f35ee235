set -o pipefail
OUT=gpurun_out/${1:-r04m}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kv -o kv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-samples 0 --no-extras --digest-batches 0 > $OUT/bench_rocprof_kv.log 2>&1 || { echo "ROCPROF KV FAILED"; tail -20 $OUT/bench_rocprof_kv.log; exit 1; }
f=$(find $OUT/prof_kv -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats_kv.csv; cut -d, -f1-4 $OUT/kernel_stats_kv.csv | cut -c1-140 | head -14
timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]); print('C4 default', d['value']/1e6, d['ms_per_step'])"
if [ -f build_exp/libnwcrypto_ldspad.so ]; then
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_ldspad.so timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_ldspad.json 2> $OUT/bench_c4_ldspad.err || { echo "C4 LDSPAD FAILED"; tail -20 $OUT/bench_c4_ldspad.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c4_ldspad.json').read().strip().splitlines()[-1]); print('C4 ldspad', d['value']/1e6, d['ms_per_step'])"
fi
exit 0
