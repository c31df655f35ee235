#!/bin/bash
# Build experimental variants of libnwcrypto.so into build_exp/ (A/B runs via NWCRYPTO_LIB=...).
# Usage: bash tools/build_variants.sh NAME "EXTRA_HIPCC_FLAGS" [NAME "FLAGS" ...]
# REBUILD="obj1.o obj2.o" limits the recompiled objects (the others are copied from the default
# build, which must be current): e.g. REBUILD="nw_kv_w20.o nw_kvs_w20.o" for a k_verify A/B at C2.
# build_exp/ is in .gpurunignore: remove that line for the call that runs the A/B.
set -e
cd "$(dirname "$0")/../narwhal_amd/csrc"
mkdir -p ../../build_exp
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=/tmp/nwv_$name; rm -rf $d; mkdir -p $d
  if [ -n "$REBUILD" ]; then
    cp -p *.o *.d $d/
    for o in $REBUILD; do rm -f $d/$o; done
  fi
  make -j8 OBJDIR=$d OUT=../../build_exp/libnwcrypto_$name.so EXTRA="$flags" > $d/build.log 2>&1
  echo built $name
done
