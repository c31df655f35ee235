set -o pipefail
OUT=gpurun_out/${1:-r04y}; mkdir -p $OUT; export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/wtrace -o w -- python3 tools/worker_leg.py > $OUT/worker_q8.json 2> $OUT/wtrace.log || { echo "TRACE FAILED"; tail -20 $OUT/wtrace.log; exit 1; }
cat $OUT/worker_q8.json | head -c 400
ls $OUT/wtrace
exit 0
