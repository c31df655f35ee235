set -o pipefail
OUT=gpurun_out/${1:-r04e}; mkdir -p $OUT
timeout -k 10 120 ./tools/sha_place 1000 1 4 > $OUT/place_g1.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/sha_place 1000 64 1 > $OUT/place_g64.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
wc -l $OUT/*.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_ranges.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/gpu_worker_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error" $OUT/gpu_worker_tests.log | head -30; tail -5 $OUT/gpu_worker_tests.log; exit 1; }
tail -2 $OUT/gpu_worker_tests.log
