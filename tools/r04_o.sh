set -o pipefail
OUT=gpurun_out/${1:-r04o}; mkdir -p $OUT; export TMPDIR=/tmp
for v in s2 s1 ldspad; do
  if [ $v = s1 ]; then A="--streams 1"; L=""; elif [ $v = ldspad ]; then A="--streams 2"; L=$PWD/build_exp/libnwcrypto_ldspad.so; else A="--streams 2"; L=""; fi
  NWCRYPTO_LIB=$L timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline $A > $OUT/bench_c4_$v.json 2> $OUT/bench_c4_$v.err || { echo "C4 $v FAILED"; tail -20 $OUT/bench_c4_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c4_$v.json').read().strip().splitlines()[-1]); print('C4 $v', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o c4 -- python3 bench.py --config C4 --steps 6 --warmup 2 --no-cpu-baseline --latency-samples 0 > $OUT/prof_c4.log 2>&1 || { echo "PROF C4 FAILED"; tail -20 $OUT/prof_c4.log; exit 1; }
f=$(find $OUT/prof_c4 -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/kernel_stats_c4.csv
for v in def fk8; do
  L=""; [ $v = fk8 ] && L=$PWD/build_exp/libnwcrypto_fk8.so
  NWCRYPTO_LIB=$L timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --latency-samples 0 > $OUT/bench_c2_$v.json 2> $OUT/bench_c2_$v.err || { echo "C2 $v FAILED"; tail -20 $OUT/bench_c2_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c2_$v.json').read().strip().splitlines()[-1]); print('C2 $v', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
exit 0
