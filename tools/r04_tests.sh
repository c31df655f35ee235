# Round 4: GPU tests, then a short C2 headline bench (no extras).  Usage: bash tools/r04_tests.sh TAG
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=15 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-extras --digest-batches 0 --cpu-seconds 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "BENCH FAILED"; tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
fi
exit 0
