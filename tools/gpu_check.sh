#!/bin/bash
# One GPU call: parity tests, a bench line, and rocprofv3 kernel-trace summaries.
#   pass 1 (prof_kv):  headline only (every k_verify launch is full size) -> agrees with the
#                      bench line's live HIP-event k_verify time
#   pass 2 (prof_all): every leg (digest overlap, MSM) -> per-kernel times of k_msm_*, k_sha512_many
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v --durations=25 --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kv -o kv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-samples 0 --no-extras --digest-batches 0 > $OUT/bench_under_rocprof_kv.log 2>&1 || { echo "ROCPROF KV FAILED"; tail -20 $OUT/bench_under_rocprof_kv.log; exit 1; }
f=$(find $OUT/prof_kv -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_kv.csv && cut -d, -f1-4 $OUT/kernel_stats_kv.csv | cut -c1-150 | head -14
if [ -z "$SKIP_PROF_ALL" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_all -o all -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --latency-samples 0 > $OUT/bench_under_rocprof_all.log 2>&1 || { echo "ROCPROF ALL FAILED"; tail -20 $OUT/bench_under_rocprof_all.log; exit 1; }
f=$(find $OUT/prof_all -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_all.csv && cut -d, -f1-4 $OUT/kernel_stats_all.csv | cut -c1-150 | head -30
f=$(find $OUT/prof_all -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && grep -E "k_sha512_many|k_verify|Kernel_Name" "$f" | cut -c1-400 > $OUT/trace_sha_verify.csv
fi
if [ -n "$TRACE_ONECALL" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof_onecall -o t -- python3 tools/one_call_trace.py > $OUT/onecall.log 2>&1 || { echo "ONECALL FAILED"; tail -20 $OUT/onecall.log; exit 1; }
grep '^{' $OUT/onecall.log
python3 tools/one_call_trace.py --analyze $OUT/prof_onecall > $OUT/onecall_anatomy.txt 2>&1; tail -12 $OUT/onecall_anatomy.txt | cut -c1-600
fi
if [ -n "$CONFIGS" ]; then
timeout -k 10 600 python3 -u tools/bench_configs.py --only $CONFIGS --cpu-seconds 0 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "CONFIGS FAILED"; tail -20 $OUT/configs.err; exit 1; }
cut -c1-400 $OUT/configs.jsonl
fi
if [ -n "$PROF_CONFIG" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg -o cfg -- python3 tools/bench_configs.py --only $PROF_CONFIG --cpu-seconds 0 --steps 3 > $OUT/prof_cfg.log 2>&1 || { echo "PROF CONFIG FAILED"; tail -20 $OUT/prof_cfg.log; exit 1; }
f=$(find $OUT/prof_cfg -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_cfg.csv && cut -d, -f1-4 $OUT/kernel_stats_cfg.csv | cut -c1-150 | head -24
fi
exit 0
