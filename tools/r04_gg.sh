# Quad-split strict uncached kernel: GPU tests of the uncached paths, latency by call size, kernel times.
set -o pipefail
OUT=gpurun_out/${1:-r04gg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_keys.py tests/test_gpu_concurrency.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python3 -u tools/strict_latency.py > $OUT/strict_latency.jsonl 2> $OUT/strict_latency.err || { echo "LATENCY FAILED"; tail -20 $OUT/strict_latency.err; exit 1; }
cat $OUT/strict_latency.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o sl -- python3 tools/strict_latency.py --samples 30 > $OUT/prof.jsonl 2> $OUT/prof.log || { echo "ROCPROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/sl_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])" | head -20
exit 0
