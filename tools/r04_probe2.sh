set -o pipefail
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 ./tools/sha_lone 3970 > $OUT/sha_lone.jsonl 2>&1 || exit 1
grep x_mode $OUT/sha_lone.jsonl | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $OUT/hf_trace -o hf -- python3 tools/host_fed_reps.py 6 > $OUT/hf_trace.log 2>&1 || { echo "HF TRACE FAILED"; tail -5 $OUT/hf_trace.log; exit 1; }
tail -1 $OUT/hf_trace.log | cut -c1-300
bash tools/r04_pmc.sh ${1:-r04h}/pmc || exit 1
exit 0
