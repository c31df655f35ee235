set -o pipefail
OUT=gpurun_out/${1:-r04x}; mkdir -p $OUT; export TMPDIR=/tmp
for v in q8a q8b q8c; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 -u tools/worker_leg.py > $OUT/worker_$v.json 2> $OUT/worker_$v.err || { echo "WORKER $v FAILED"; tail -20 $OUT/worker_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/worker_$v.json')); w=d['windows']; print('$v', {k:(round(x['batches_per_s']), round(x['p50_latency_ms'],1)) for k,x in w.items()})"
done
exit 0
