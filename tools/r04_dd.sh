set -o pipefail
OUT=gpurun_out/${1:-r04dd}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3; do for v in 1 3; do
  timeout -k 10 200 python3 -u bench.py --streams $v --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 > $OUT/bench_c2_s${v}_$r.json 2> $OUT/bench_c2_s${v}_$r.err || { echo "C2 s$v FAILED"; tail -20 $OUT/bench_c2_s${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c2_s${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2 s$v rep $r', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(r['frac'],3), round(r['avg_launch_ms'],4), round(r['isolated']['frac'],3))"
done; done
exit 0
