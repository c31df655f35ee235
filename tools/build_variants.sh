#!/bin/bash
# Build experimental variants of libnwcrypto.so into build_exp/ (A/B runs via NWCRYPTO_LIB=...).
# Usage: bash tools/build_variants.sh NAME "EXTRA_HIPCC_FLAGS" [NAME "FLAGS" ...]
set -e
cd "$(dirname "$0")/../narwhal_amd/csrc"
mkdir -p ../../build_exp
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=/tmp/nwv_$name; mkdir -p $d
  make -j8 OBJDIR=$d OUT=../../build_exp/libnwcrypto_$name.so EXTRA="$flags" > $d/build.log 2>&1
  echo built $name
done
