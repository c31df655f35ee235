#!/bin/bash
# A/B of runtime knobs (environment variables read by libnwcrypto) on the C2 bench (GPU box).
# Usage: bash tools/ab_env.sh TAG "NAME=VAR=VALUE" ...   e.g.  bash tools/ab_env.sh ab_fk fk4=NW_FK=4 fk8=NW_FK=8
set -o pipefail
OUT=gpurun_out/${1:-ab_env}
shift
mkdir -p $OUT
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras ${BENCH_ARGS:-}"
for rep in 1 2; do
for spec in default "$@"; do
  name=${spec%%=*}
  if [ "$spec" = default ]; then
    timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "FAIL $name"; tail -5 $OUT/$name.$rep.err; exit 1; }
  else
    kv=${spec#*=}
    env "$kv" timeout -k 10 240 python bench.py $ARGS > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "FAIL $name"; tail -5 $OUT/$name.$rep.err; exit 1; }
  fi
  python -c "import json; d=json.load(open('$OUT/$name.$rep.json')); print('%-16s %8.1f Msig/s  %.4f ms/step  k_verify %.3f ms' % ('$name', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms']))"
done
done
