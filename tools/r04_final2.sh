set -o pipefail
OUT=gpurun_out/${1:-r04final2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(r['frac'],3), r['avg_launch_ms'], r.get('isolated',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kv -o kv -- python3 bench.py --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 > $OUT/bench_kv.json 2> $OUT/prof_kv.log || { echo "ROCPROF KV FAILED"; tail -20 $OUT/prof_kv.log; exit 1; }
python3 tools/roofline_rocprof.py $OUT/prof_kv/kv_kernel_trace.csv --bench $OUT/bench_kv.json --skip 2 --take 10 > $OUT/roofline_rocprof.json && cat $OUT/roofline_rocprof.json
for v in def fk32 def2; do
  L=""; [ $v = fk32 ] && L=$PWD/build_exp/libnwcrypto_fk32.so
  NWCRYPTO_LIB=$L timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 > $OUT/bench_c2_$v.json 2> $OUT/bench_c2_$v.err || { echo "C2 $v FAILED"; tail -20 $OUT/bench_c2_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c2_$v.json').read().strip().splitlines()[-1]); print('C2 $v', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
exit 0
