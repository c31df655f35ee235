set -o pipefail
OUT=gpurun_out/${1:-r04q}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for v in excl noexcl excl2 noexcl2; do
  L=""; case $v in noexcl*) L=$PWD/build_exp/libnwcrypto_noexcl.so;; esac
  NWCRYPTO_LIB=$L timeout -k 10 400 python3 -u bench.py --config C4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_$v.json 2> $OUT/bench_c4_$v.err || { echo "C4 $v FAILED"; tail -20 $OUT/bench_c4_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c4_$v.json').read().strip().splitlines()[-1]); print('C4 $v', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))"
done
timeout -k 10 300 rocprofv3 --hip-runtime-trace --memory-copy-trace --kernel-trace --output-format csv -d $OUT/hf_trace -o hf -- python3 tools/host_fed_reps.py 8 trace > $OUT/hf_trace.log 2>&1 || { echo "HF TRACE FAILED"; tail -20 $OUT/hf_trace.log; exit 1; }
ls $OUT/hf_trace
exit 0
