set -o pipefail
export PMC_CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-samples 0 --no-extras --digest-batches 0"
export PMC_PASSES=3
timeout -k 10 900 bash tools/gpu_pmc.sh ${1:-r04pmc3} "k_finish" || exit 1
exit 0
