set -o pipefail
OUT=gpurun_out/${1:-r04k}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 ./tools/slow_probe > $OUT/slow_probe.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 240 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep -E '"kernel"|split2_rep' $OUT/sha_lone.jsonl | cut -c1-220
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('per_cycle',{}).get('frac_per_cycle'))
g=d['digest']; print('single_chain', g['single_chain']); print('c4_share', g['c4_share']['kernel_ms'])
print('header', d['latency']['header_digest_6667_parents'])
print('worker', json.dumps(d['worker_digest'])[:900])
print('host_fed', d['host_fed']['ms_reps'], d['host_fed']['fresh_buffers']['ms_reps'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $OUT/hf_trace -o hf -- python3 tools/host_fed_reps.py 30 > $OUT/hf_trace.log 2>&1 || { echo "HF TRACE FAILED"; tail -5 $OUT/hf_trace.log; exit 1; }
grep '^{' $OUT/hf_trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced host_fed', [round(p['ms'],2) for p in d['passes']])"
exit 0
