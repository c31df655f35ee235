#!/bin/bash
# Per-kernel rocprofv3 averages of the default build vs every build_exp/*.so variant on one bench
# config.  Usage: KRE='k_finish|k_verify' BENCH_ARGS='--config C4 --steps 6' bash tools/ab_kernel_stats.sh TAG
set -o pipefail
shopt -s nullglob
OUT=gpurun_out/${1:-abk}
mkdir -p $OUT
export TMPDIR=/tmp
KRE=${KRE:-k_finish|k_verify}
ARGS="--steps 10 --warmup 2 --c4-steps 0 --no-cpu-baseline --digest-batches 0 --latency-samples 0 --no-extras ${BENCH_ARGS:-}"
for lib in default build_exp/*.so; do
  name=$(basename $lib .so)
  if [ "$lib" = default ]; then unset NWCRYPTO_LIB; else export NWCRYPTO_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o k -- \
    python3 bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; exit 1; }
  f=$(find $OUT/$name -name 'k_kernel_stats.csv' | head -1)
  python3 - "$f" "$OUT/$name.json" "$name" "$KRE" <<'EOF'
import csv, json, re, sys
f, j, name, kre = sys.argv[1:]
d = json.load(open(j))
row = ["%-22s %7.1f M/s %7.3f ms/step" % (name, d["value"] / 1e6, d["ms_per_step"])]
for r in csv.DictReader(open(f)):
    if re.search(kre, r["Name"]):
        row.append("%s %.1f us" % (re.sub(r"\(.*", "", r["Name"])[-28:], float(r["AverageNs"]) / 1e3))
print("  ".join(row))
EOF
done
