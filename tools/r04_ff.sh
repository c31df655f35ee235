set -o pipefail
OUT=gpurun_out/${1:-r04ff}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 400 python3 -u tools/bench_configs.py --only W,C3 --cpu-seconds 0 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "CONFIGS FAILED"; tail -20 $OUT/configs.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); print(d['config'], round(d['sigs_per_s']/1e6,1), d.get('key_window'), round(d.get('ms_per_step', d.get('ms_per_batch', 0)),3))"
exit 0
