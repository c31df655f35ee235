set -o pipefail
OUT=gpurun_out/${1:-r04bb}; mkdir -p $OUT; export TMPDIR=/tmp
for s in 2 3 2b 3b; do
  n=${s%b}
  timeout -k 10 400 python3 -u tools/bench_configs.py --only C5,C3 --cpu-seconds 0 --streams $n > $OUT/configs_s$s.jsonl 2> $OUT/configs_s$s.err || { echo "CONFIGS $s FAILED"; tail -20 $OUT/configs_s$s.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/configs_s$s.jsonl'):
    d=json.loads(l); print('streams $s', d['config'], round(d['sigs_per_s']/1e6,1), 'serial', round(d['sigs_per_s_serial']/1e6,1), d['parity'].get('mismatches'), d['parity'].get('strict_mismatches'))"
done
exit 0
