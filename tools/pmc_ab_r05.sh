#!/bin/bash
# k_verify shader cycles per C2 launch (PMC GRBM_GUI_ACTIVE: clock-independent) for library / env
# variants, interleaved in one GPU call.  Wall time on this pool moves +-5% with the power-managed
# clock; cycles do not.
#   bash tools/pmc_ab_r05.sh OUTTAG "tag1 ENV=VAL ..." "tag2 NWCRYPTO_LIB=build_exp/x.so" "tag3 --bench-arg=v" ...
# Summary: python3 tools/pmc_ab_summary.py gpurun_out/OUTTAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?usage: pmc_ab_r05.sh OUTTAG "tag [ENV=VAL ...]" ...}
shift
mkdir -p "$OUT"
CMD="python3 bench.py --steps 4 --warmup 1 --c4-steps 0 --no-cpu-baseline --latency-samples 0 --digest-batches 0 --no-extras"
for spec in "$@"; do
  set -- $spec
  tag=$1; shift
  envs=(X=1); extra=""
  for t in "$@"; do case $t in --*) extra="$extra $t" ;; *) envs+=("$t") ;; esac; done
  env "${envs[@]}" timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU \
    --kernel-include-regex "k_verify<" --output-format csv -d "$OUT/$tag" -o p -- $CMD $extra > "$OUT/$tag.log" 2>&1 \
    || { echo "FAIL $tag"; tail -3 "$OUT/$tag.log"; exit 1; }
  echo "ok $tag"
done
