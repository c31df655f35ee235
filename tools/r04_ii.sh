# Kernel breakdown of single-certificate calls (tools/latency_probe.py at C2 / C3 sizes) after k_finish<true>.
set -o pipefail
OUT=gpurun_out/${1:-r04ii}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o lat -- python3 tools/latency_probe.py --samples 100 --only 100,1000 > $OUT/latency.jsonl 2> $OUT/prof.log || { echo "ROCPROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
cat $OUT/latency.jsonl | cut -c1-400
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/lat_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'])" | head -24
exit 0
