#!/bin/bash
# A/B runtime tunables (environment variables read by libnwcrypto) on the C2 bench (GPU box).
# Usage: bash tools/ab_env.sh TAG "ENV1" "ENV2" ...   e.g. "NW_PIPE=1" "NW_PIPE=0.45,0.45,0.1"
set -o pipefail
OUT=gpurun_out/${1:-abenv}; shift
mkdir -p $OUT
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras ${BENCH_ARGS:-}"
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 240 python bench.py $ARGS > $OUT/v$i.$rep.json 2> $OUT/v$i.$rep.err || { echo "FAIL [$envs]"; tail -5 $OUT/v$i.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/v$i.$rep.json')); print('%-40s %8.1f Msig/s  %.3f ms/step  k_verify %.3f ms x %d' % ('$envs', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches']))"
  done
done
