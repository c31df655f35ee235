#!/bin/bash
# Calibrate SQ_THREAD_CYCLES_VALU units on a kernel that is VALU-bound by construction
# (tools/valu_peak k_mad_u64_u32: 16 independent MAD chains per lane, no memory traffic).
set -o pipefail
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/valu_peak > $OUT/valu_peak.jsonl 2>&1 || { echo "valu_peak failed"; exit 1; }
cat $OUT/valu_peak.jsonl
timeout -s KILL 60 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex "k_mad_u64_u32|k_mul_lo" --output-format csv -d $OUT/c -o c -- ./tools/valu_peak > $OUT/calib.log 2>&1 || { echo "calib pmc failed"; tail -5 $OUT/calib.log; exit 1; }
f=$(find $OUT/c -name '*counter_collection.csv' | head -1); cp "$f" $OUT/calib_pmc.csv
