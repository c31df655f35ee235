#!/bin/bash
# Worker-digest bimodality vs NUMA placement: the worker leg bound to each
# socket's CPUs in turn (first-touch puts the pinned staging buffers on that socket's memory), and the
# GPU's own NUMA node from sysfs.  Usage (GPU box): bash tools/numa_probe.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-numa}
mkdir -p "$OUT"
for d in /sys/class/drm/card*/device; do
  [ -f "$d/numa_node" ] && echo "$d numa_node=$(cat $d/numa_node) $(cat $d/uevent 2>/dev/null | grep PCI_SLOT_NAME)"
done > "$OUT/gpu_numa.txt"
cat "$OUT/gpu_numa.txt"
for node in 0 1 0 1; do
  cpus=$( [ $node = 0 ] && echo 0-63 || echo 64-127 )
  timeout -k 10 200 taskset -c $cpus python3 tools/worker_leg.py > "$OUT/wl_node$node.$RANDOM.json" 2> "$OUT/wl_node$node.err" || { tail -5 "$OUT/wl_node$node.err"; exit 1; }
done
for f in "$OUT"/wl_node*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); w=d['windows']; print('$f', {k: round(v['batches_per_s']) for k, v in w.items()}, 'p50', round(w['1250']['p50_latency_ms'], 1))"
done
