# Fresh PMC passes on the closing build (C2 k_verify): SQ groups, FETCH_SIZE, WRITE_SIZE, one per run.
set -o pipefail
export PMC_CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-samples 0 --no-extras --digest-batches 0"
export PMC_PASSES=4
timeout -k 10 900 bash tools/gpu_pmc.sh ${1:-r04pmc2} "k_verify" || exit 1
exit 0
