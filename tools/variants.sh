#!/bin/bash
# Build variant copies of libnemohip with extra compile definitions and/or
# replaced source files, for A/B kernel experiments on the GPU box
# (NEMO_LIB=var/NAME/libnemohip.so python bench.py ...).
#   tools/variants.sh NAME "-DFOO=1 -DBAR=2" [NAME2 "..."]
#   OVERLAY="k_load.hip=/tmp/alt.hip" tools/variants.sh NAME ""
# Output: var/NAME/libnemohip.so (git-ignored; travels with gpurun; objects under build/).
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  out=build/variants/$name
  rm -rf $out; mkdir -p $out/src var/$name
  cp nemo_amd/csrc/* $out/src/
  for ov in $OVERLAY; do cp "${ov#*=}" "$out/src/${ov%%=*}"; done
  sed -i 's|#include "../../include/nemohip.h"|#include "'"$PWD"'/include/nemohip.h"|' $out/src/*.h $out/src/*.hip $out/src/*.cpp 2>/dev/null || true
  objs=""
  for f in $out/src/*.hip; do
    o=$out/$(basename $f .hip).o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value $defs -c -o $o $f &
    objs="$objs $o"
  done
  for f in $out/src/*.cpp; do
    o=$out/$(basename $f .cpp).host.o
    g++ -O3 -std=c++17 -fPIC -pthread -Wall $defs -c -o $o $f &
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o var/$name/libnemohip.so $objs -pthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built var/$name/libnemohip.so ($defs ${OVERLAY})"
done
