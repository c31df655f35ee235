#!/bin/bash
# A/B the libnwcrypto variants in build_exp/ against the default build on the C2 bench (GPU box).
set -o pipefail
shopt -s nullglob
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
ARGS="--steps 20 --warmup 3 --c4-steps 0 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras ${BENCH_ARGS:-}"
for rep in 1 2; do
for lib in default build_exp/*.so; do
  name=$(basename $lib .so)
  if [ "$lib" = default ]; then
    timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "FAIL $name"; tail -5 $OUT/$name.$rep.err; exit 1; }
  else
    NWCRYPTO_LIB=$PWD/$lib timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "FAIL $name"; tail -5 $OUT/$name.$rep.err; exit 1; }
  fi
  python -c "import json,sys; d=json.load(open('$OUT/$name.$rep.json')); print('%-28s %8.1f Msig/s  k_verify %.3f ms' % ('$name', d['value']/1e6, d['roofline']['avg_launch_ms']))"
done
done
