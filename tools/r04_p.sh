set -o pipefail
OUT=gpurun_out/${1:-r04p}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3; do for v in 1 2; do
  timeout -k 10 200 python3 -u bench.py --streams $v --no-extras --no-cpu-baseline --latency-samples 0 > $OUT/bench_c2_s${v}_$r.json 2> $OUT/bench_c2_s${v}_$r.err || { echo "C2 s$v FAILED"; tail -20 $OUT/bench_c2_s${v}_$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c2_s${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C2 s$v rep $r', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), r.get('isolated') and round(r['isolated']['avg_launch_ms'],4))"
done; done
timeout -k 10 300 python3 -u tools/host_fed_reps.py 20 > $OUT/host_fed_reps.json 2> $OUT/host_fed_reps.err || { echo "HOSTFED FAILED"; tail -20 $OUT/host_fed_reps.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/host_fed_reps.json')); print('host_fed median', round(d['median_ms'],2), 'slow', [(p['pass'], round(p['ms'],1)) for p in d['slow_passes']], 'fresh', [round(x,1) for x in d['fresh_passes_ms']])"
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('C2 full', d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('isolated')); print(json.dumps(d['worker_digest'])[:900]); print(json.dumps(d['host_fed'])[:400])"
exit 0
