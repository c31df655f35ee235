set -o pipefail
OUT=gpurun_out/${1:-r04f}; mkdir -p $OUT
timeout -k 10 180 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep x_mode $OUT/sha_lone.jsonl | cut -c1-260
