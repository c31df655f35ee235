# k_finish<true> inversion A/B for single-certificate calls: constant-time (default, > 8 signatures)
# vs variable-time up to 65,536 signatures (build_exp/libnwcrypto_var.so).
set -o pipefail
OUT=gpurun_out/${1:-r04jj}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/def -o lat -- python3 tools/latency_probe.py --samples 100 --only 100,1000 > $OUT/def.jsonl 2> $OUT/def.log || { echo "DEF FAILED"; tail -20 $OUT/def.log; exit 1; }
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_var.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/var -o lat -- python3 tools/latency_probe.py --samples 100 --only 100,1000 > $OUT/var.jsonl 2> $OUT/var.log || { echo "VAR FAILED"; tail -20 $OUT/var.log; exit 1; }
for v in def var; do
  echo "== $v"; cut -c1-200 $OUT/$v.jsonl
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$v/lat_kernel_stats.csv')):
    if 'finish' in r['Name'] or 'split' in r['Name']: print(r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'])"
done
exit 0
