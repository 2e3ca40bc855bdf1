#!/bin/bash
# Build variant copies of libnemohip with extra compile definitions, for A/B
# kernel experiments on the GPU box (NEMO_LIB=<path> python bench.py ...).
#   tools/variants.sh NAME "-DFOO=1 -DBAR=2" [NAME2 "..."]
# Output: var/NAME/libnemohip.so (git-ignored; travels with gpurun; objects under build/).
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  out=build/variants/$name
  mkdir -p $out
  objs=""
  for f in nemo_amd/csrc/*.hip; do
    o=$out/$(basename $f .hip).o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value $defs -c -o $o $f &
    objs="$objs $o"
  done
  for f in nemo_amd/csrc/*.cpp; do
    o=$out/$(basename $f .cpp).host.o
    g++ -O3 -std=c++17 -fPIC -pthread -Wall $defs -c -o $o $f &
    objs="$objs $o"
  done
  wait
  mkdir -p var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o var/$name/libnemohip.so $objs -pthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built var/$name/libnemohip.so ($defs)"
done
