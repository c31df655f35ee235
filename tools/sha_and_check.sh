# One GPU call: the lone-chain SHA-512 placement probe (tools/sha_lone), then tools/gpu_check.sh
# with the C3/C4/C5 timings and a C5 kernel trace.  Usage: bash tools/sha_and_check.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 ./tools/sha_lone 4000 > gpurun_out/$TAG/sha_lone.jsonl 2>&1 && grep -E "split2_rep|k_sha512_split2" gpurun_out/$TAG/sha_lone.jsonl || exit 1
SKIP_PROF_ALL=${SKIP_PROF_ALL-1} CONFIGS=${CONFIGS-C3,C4,C5} PROF_CONFIG=${PROF_CONFIG-C5} bash tools/gpu_check.sh $TAG
