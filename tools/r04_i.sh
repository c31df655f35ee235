set -o pipefail
OUT=gpurun_out/${1:-r04i}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep copies $OUT/sha_lone.jsonl
timeout -k 10 300 python3 -u tools/host_fed_reps.py 12 > $OUT/host_fed_reps.json 2> $OUT/host_fed_reps.err || { echo "HOSTFED FAILED"; tail -5 $OUT/host_fed_reps.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/host_fed_reps.json')); print('host_fed', round(d['median_ms'],3), [round(p['ms'],2) for p in d['passes']], 'fresh', [round(x,2) for x in d['fresh_passes_ms']])"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
exit 0
