# VALU instructions and cycles of the quad / lane strict kernels (k_verify_var<true> at 1 signature,
# <false> at 4,097) and k_finish: two PMC passes over tools/strict_latency.py.
set -o pipefail
export PMC_CMD="python3 tools/strict_latency.py --sizes 1,4097 --samples 5"
export PMC_PASSES=2
timeout -k 10 400 bash tools/gpu_pmc.sh ${1:-r04pmc5} "k_verify_var|k_finish" || exit 1
exit 0
