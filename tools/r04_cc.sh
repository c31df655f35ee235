set -o pipefail
OUT=gpurun_out/${1:-r04cc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for s in 3 2; do
  timeout -k 10 400 python3 -u tools/bench_configs.py --only C5,C3 --cpu-seconds 0 --streams $s > $OUT/configs_s$s.jsonl 2> $OUT/configs_s$s.err || { echo "CONFIGS $s FAILED"; tail -20 $OUT/configs_s$s.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/configs_s$s.jsonl'):
    d=json.loads(l); print('streams $s', d['config'], round(d['sigs_per_s']/1e6,1), 'serial', round(d['sigs_per_s_serial']/1e6,1), d['parity'].get('mismatches'), d['parity'].get('strict_mismatches'))"
done
exit 0
