#!/bin/bash
# Build the working tree's liballl.so with extra compile flags into build/ab/liballl_<name>.so
# (A/B timing through ALLL_LIB_AB; the in-tree library is left alone).
# usage: bash tools/build_variant.sh <name> "<flags>"
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
D=$(mktemp -d /tmp/abv.XXXX)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ialllsatisfiabilitysolver_amd/csrc -I/opt/rocm/include $FLAGS"
for f in $(cd alllsatisfiabilitysolver_amd/csrc && ls *.hip *.cpp); do
  /opt/rocm/bin/hipcc $F -c -o $D/${f%.*}.o alllsatisfiabilitysolver_amd/csrc/$f &
done
wait
mkdir -p build/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/liballl_$NAME.so $D/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $D
ls -la build/ab/liballl_$NAME.so
