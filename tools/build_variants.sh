#!/bin/bash
# Build alternative libphc_hip builds for A/B runs: tools/build_variants.sh name "EXTRA flags" [name "flags" ...]
# -> puffer-phc_amd/lib/libphc_hip_<name>.so (objects under csrc/build/<name>)
set -eu
cd "$(dirname "$0")/../puffer-phc_amd/csrc"
while [ $# -ge 2 ]; do
  make -s -j8 OBJDIR=build/$1 OUT=../lib/libphc_hip_$1.so EXTRA="$2"
  echo "built libphc_hip_$1.so ($2)"
  shift 2
done
