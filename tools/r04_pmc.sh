# Round 4: clock-normalised VALU peak.  The v_mad_u64_u32 microbenchmark and a C2 bench, each under
# one PMC pass with GRBM_GUI_ACTIVE (+ VALU counts), so peak and k_verify are both per cycle.
set -o pipefail
OUT=gpurun_out/${1:-r04pmc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 60 ./tools/valu_peak > $OUT/valu_peak.jsonl 2>&1 || exit 1
cat $OUT/valu_peak.jsonl
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 --kernel-trace --output-format csv -d $OUT/peak -o peak -- ./tools/valu_peak > $OUT/peak_pmc.log 2>&1 || { echo "PMC peak failed"; tail -5 $OUT/peak_pmc.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT64 --kernel-include-regex "k_verify|k_finish" --output-format csv -d $OUT/kv -o kv -- python3 bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline --digest-batches 0 --latency-samples 0 > $OUT/kv_pmc.log 2>&1 || { echo "PMC kv failed"; tail -5 $OUT/kv_pmc.log; exit 1; }
ls $OUT/peak $OUT/kv
exit 0
