#!/bin/bash
# host_fed stalls: tools/host_fed_sweep.py under runtime environment variants and library variants
# (build_exp/, NWCRYPTO_LIB).  Usage: bash tools/env_sweep.sh TAG "VAR=VAL[,VAR=VAL]|LIB" ...
set -o pipefail
TAG=${1:-envsweep}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for spec in "$@"; do
  envs=${spec%%|*}; lib=""; [ "$spec" != "$envs" ] && lib=${spec#*|}
  L=""; [ -n "$lib" ] && L=$PWD/build_exp/libnwcrypto_$lib.so
  env ${envs//,/ } NWCRYPTO_LIB=$L timeout -k 10 120 python3 -u tools/host_fed_sweep.py ${SHAPES:-16x8} > $OUT/o.tmp 2>&1 \
    || { echo "FAIL $spec"; tail -5 $OUT/o.tmp; exit 1; }
  grep '^{' $OUT/o.tmp | sed "s/^/$spec /" | tee -a $OUT/sweep.txt | cut -c1-240
done
