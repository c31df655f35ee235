#!/bin/bash
# One GPU call: parity tests, a bench line, and a rocprofv3 kernel-trace summary of the same bench.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o $TAG -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --latency-samples 0 ${BENCH_ARGS:-} > $OUT/bench_under_rocprof.log 2>&1 || { echo "ROCPROF FAILED"; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv && cut -d, -f1-4 $OUT/kernel_stats.csv | cut -c1-150 | head -14
exit 0
