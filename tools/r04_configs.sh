# Round 4: the north-star config C4 (and C3) through bench.py on one GPU, with the host baseline,
# plus a rocprofv3 kernel-trace summary of the C4 step.  Usage (via gpurun): bash tools/r04_configs.sh TAG
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
cut -c1-1500 $OUT/bench_c4.json
timeout -k 10 300 python3 -u bench.py --config C3 --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "C3 FAILED"; tail -20 $OUT/bench_c3.err; exit 1; }
cut -c1-600 $OUT/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 5 --warmup 1 --no-cpu-baseline --latency-samples 0 > $OUT/bench_c4_rocprof.log 2>&1 || { echo "ROCPROF C4 FAILED"; tail -20 $OUT/bench_c4_rocprof.log; exit 1; }
f=$(find $OUT/prof_c4 -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/kernel_stats_c4.csv && cut -d, -f1-4 $OUT/kernel_stats_c4.csv | cut -c1-150 | head -24
exit 0
