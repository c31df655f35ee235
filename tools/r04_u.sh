set -o pipefail
OUT=gpurun_out/${1:-r04u}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_$r.json 2> $OUT/bench_c4_$r.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c4_$r.json').read().strip().splitlines()[-1]); print('C4', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3), d['config']['key_window'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 6 --warmup 2 --no-cpu-baseline --latency-samples 0 > $OUT/prof_c4.log 2>&1 || { echo "PROF C4 FAILED"; tail -20 $OUT/prof_c4.log; exit 1; }
f=$(find $OUT/prof_c4 -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats_c4.csv
exit 0
