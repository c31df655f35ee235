#!/bin/bash
# Build experimental variants of libnwcrypto.so into build_exp/ (A/B runs via NWCRYPTO_LIB=...).
# Usage: bash tools/build_variants.sh NAME "EXTRA_HIPCC_FLAGS" [NAME "FLAGS" ...]
set -e
cd "$(dirname "$0")/../narwhal_amd/csrc"
mkdir -p ../../build_exp
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=/tmp/nwv_$name; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -c nw_kernels.hip -o $d/k.o &
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -x hip -c nw_api.cpp -o $d/a.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/k.o $d/a.o -o ../../build_exp/libnwcrypto_$name.so
  echo built $name
done
