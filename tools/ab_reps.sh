#!/bin/bash
# Interleaved A/B of the default build against the build_exp/ variants, 4 reps of a 40-step C2 bench
# each (launch-to-launch clock variation makes 2-rep comparisons of ~1% effects unreliable).
set -o pipefail
OUT=gpurun_out/${1:-ab_reps}
mkdir -p $OUT
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras ${BENCH_ARGS:-}"
for rep in 1 2 3 4; do
for lib in default build_exp/*.so; do
  name=$(basename $lib .so)
  if [ "$lib" = default ]; then timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2>/dev/null || exit 1
  else NWCRYPTO_LIB=$PWD/$lib timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2>/dev/null || exit 1; fi
  python -c "import json; d=json.load(open('$OUT/$name.$rep.json')); print('%-24s %8.1f Msig/s  %.4f ms/step  k_verify %.4f ms' % ('$name', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms']))"
done; done
