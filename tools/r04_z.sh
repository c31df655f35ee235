set -o pipefail
OUT=gpurun_out/${1:-r04z}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -q -x --timeout 200 --timeout-method thread > $OUT/gpu_worker_tests.log 2>&1 || { echo "WORKER TESTS FAILED"; tail -15 $OUT/gpu_worker_tests.log; exit 1; }
tail -1 $OUT/gpu_worker_tests.log
for v in def fk8b def2 fk8b2; do
  L=""; case $v in fk8b*) L=$PWD/build_exp/libnwcrypto_fk8b.so;; esac
  NWCRYPTO_LIB=$L timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 > $OUT/bench_c2_$v.json 2> $OUT/bench_c2_$v.err || { echo "C2 $v FAILED"; tail -20 $OUT/bench_c2_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c2_$v.json').read().strip().splitlines()[-1]); print('C2 $v', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
NWCRYPTO_LIB=$PWD/build_exp/libnwcrypto_fk8b.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python3 bench.py --no-extras --no-cpu-baseline --latency-samples 0 --digest-batches 0 --steps 5 > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); grep -E "k_finish|k_verify<" $f | cut -c1-120
exit 0
