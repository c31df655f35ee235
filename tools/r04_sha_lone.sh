set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 ./tools/sha_lone_old 3970 > $OUT/sha_lone_old.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/sha_lone 3970 > $OUT/sha_lone_new.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/sha_lone_old 3970 > $OUT/sha_lone_old2.jsonl 2>&1 || exit 1
timeout -k 10 120 ./tools/sha_lone 3970 > $OUT/sha_lone_new2.jsonl 2>&1 || exit 1
cat $OUT/sha_lone_old.jsonl $OUT/sha_lone_new.jsonl | cut -c1-220
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $OUT/pmc_new -o p -- ./tools/sha_lone 3970 > $OUT/pmc_new.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $OUT/pmc_old -o p -- ./tools/sha_lone_old 3970 > $OUT/pmc_old.log 2>&1 || exit 1
exit 0
