# k_sha512_split2 cycles in the C4 step (under k_verify load) vs alone (bench digest leg's C4 share)
set -o pipefail
OUT=gpurun_out/${1:-r04pmc4}; mkdir -p $OUT; export TMPDIR=/tmp
CTRS="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "k_sha512" --output-format csv -d $OUT/c4 -o c4 -- python3 bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --latency-samples 0 > $OUT/c4.log 2>&1 || { echo "PMC C4 failed"; tail -5 $OUT/c4.log; exit 1; }
f=$(find $OUT/c4 -name '*counter_collection.csv' | head -1); cp "$f" $OUT/pmc_c4.csv
timeout -s KILL 240 rocprofv3 --pmc $CTRS --kernel-include-regex "k_sha512" --output-format csv -d $OUT/alone -o alone -- python3 tools/worker_leg.py > $OUT/alone.log 2>&1 || { echo "PMC alone failed"; tail -5 $OUT/alone.log; exit 1; }
f=$(find $OUT/alone -name '*counter_collection.csv' | head -1); cp "$f" $OUT/pmc_alone.csv
exit 0
