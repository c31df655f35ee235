#!/bin/bash
# Worker-digest bimodality probe: the worker_digest leg in 3 separate
# processes, each under rocprofv3 kernel + memory-copy traces (no PMC), then a per-process
# timeline of the WINDOW-1250 submissions: digest kernels (queue, start, end, workgroups) and H2D
# copies.  Usage (GPU box): bash tools/worker_trace.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-wtrace}
mkdir -p "$OUT"
export TMPDIR=/tmp
# PREWARM="a b c": one traced process per value (tools/worker_leg.py --prewarm)
k=0
for pw in ${PREWARM:-0 0 0}; do
  k=$((k + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/wl_$k" -o wl -- \
    python3 tools/worker_leg.py --prewarm "$pw" > "$OUT/wl_$k.json" 2> "$OUT/wl_$k.err" || { echo "worker leg $k FAILED"; tail -5 "$OUT/wl_$k.err"; exit 1; }
  python3 tools/worker_trace_summary.py "$OUT/wl_$k" "$OUT/wl_$k.json" > "$OUT/wl_$k.summary.txt" || exit 1
  head -9 "$OUT/wl_$k.summary.txt"
done
