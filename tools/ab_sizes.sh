#!/bin/bash
# Batch-size sweep of the C2 step (per-signature throughput vs certificate count): wave-quantization
# check for k_verify (3,072 wave slots on MI355X at 3 waves per SIMD).
set -o pipefail
OUT=gpurun_out/${1:-ab_sizes}; shift
mkdir -p $OUT
for rep in 1 2; do
for c in "$@"; do
  timeout -k 10 240 python bench.py --certs $c --steps 30 --warmup 5 --c4-steps 0 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras > $OUT/c$c.$rep.json 2>/dev/null || { echo "FAIL $c"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c$c.$rep.json')); n=$c*67; print('certs %6d sigs %8d waves %6d  %8.1f Msig/s  k_verify %.4f ms  ns/sig %.4f' % ($c, n, (n+63)//64, d['value']/1e6, d['roofline']['avg_launch_ms'], d['roofline']['avg_launch_ms']*1e6/n))"
done; done
