#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only — never combined with other traces)
# over a short bench run.  Usage: bash tools/gpu_pmc.sh TAG [kernel-regex]
set -o pipefail
TAG=${1:-pmc}
RE=${2:-k_verify|k_finish|k_sha512}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 bench.py --steps 2 --warmup 1 --c4-steps 0 --no-cpu-baseline --latency-samples 0 ${BENCH_ARGS:-}"}
NPASS=${PMC_PASSES:-5}   # first N counter groups only
FIRST=${PMC_FIRST:-1}    # skip the groups before this one
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  [ $i -gt $NPASS ] && break
  [ $i -lt $FIRST ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$RE" --output-format csv -d $OUT/p$i -o p$i -- $CMD > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && cp "$f" $OUT/pmc_pass$i.csv
done
ls $OUT
